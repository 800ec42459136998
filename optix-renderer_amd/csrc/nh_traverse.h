// BVH traversal for gfx950: BVH::rayIntersect (src/utils/bvh.cpp:402-460) semantics on
// a GPU node layout.
//
// Layout (HBM, built by nh_api.hip from the reference's node array):
//   inner node (64 B) = 4 x float4:
//     n0 = (L.min.xyz, L.max.x)  n1 = (L.max.yz, R.min.xy)  n2 = (R.min.z, R.max.xyz)
//     n3 = (int L.ref, int R.ref, 0, 0)   ref >= 0: inner node, ref < 0: leaf ~ref
//   leaf table: int2 (start, count) into the primitive array
//   primitive (48 B, in the reference's m_indices order) = 3 x float4:
//     triangle: (p0, local face) (p1, shape) (p2, 0) -- the vertices themselves, so
//               setHitInformation needs no index/vertex fetches for the hit point
//     sphere:   (center, radius) (0, shape) (0, 1)
// Child boxes live in the parent, so one 64-B fetch tests both children; the
// reference tests a node's own box when it is visited, which is the same set of
// tests. Deferred children carry their slab entry distance and are re-checked against
// the current maxt when popped -- exactly the reference's visit-time test, whose
// other terms do not depend on maxt.
//
// Two visit orders:
//   REFERENCE: left child first (the reference's order);
//   ORDERED:   nearer child first.
// Both return the reference's answer: the smallest t; among equal t the primitive
// latest in left-first DFS order, which is the largest leaf-order position k (the
// reference accepts t <= maxt, so a later equal-t primitive overwrites).
#pragma once
#include "nh_device.h"

namespace nhd {

struct Hit {
    float t, u, v;
    int k;  // leaf-order primitive position
};

struct TravStats {
    uint32_t nodes, boxes, prims;
};

// BoundingBox::rayIntersect (bbox.h:336-363); returns the entry distance in near_out
NHD bool box_test(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, F3 o, F3 d, F3 r, float mint,
                  float maxt, float &near_out) {
    float near_t = -INFINITY, far_t = INFINITY;
    if (d.x == 0) {
        if (o.x < mnx || o.x > mxx) return false;
    } else {
        float t1 = (mnx - o.x) * r.x, t2 = (mxx - o.x) * r.x;
        if (t1 > t2) { float tmp = t1; t1 = t2; t2 = tmp; }
        near_t = e_max(t1, near_t);
        far_t = e_min(t2, far_t);
        if (!(near_t <= far_t)) return false;
    }
    if (d.y == 0) {
        if (o.y < mny || o.y > mxy) return false;
    } else {
        float t1 = (mny - o.y) * r.y, t2 = (mxy - o.y) * r.y;
        if (t1 > t2) { float tmp = t1; t1 = t2; t2 = tmp; }
        near_t = e_max(t1, near_t);
        far_t = e_min(t2, far_t);
        if (!(near_t <= far_t)) return false;
    }
    if (d.z == 0) {
        if (o.z < mnz || o.z > mxz) return false;
    } else {
        float t1 = (mnz - o.z) * r.z, t2 = (mxz - o.z) * r.z;
        if (t1 > t2) { float tmp = t1; t1 = t2; t2 = tmp; }
        near_t = e_max(t1, near_t);
        far_t = e_min(t2, far_t);
        if (!(near_t <= far_t)) return false;
    }
    near_out = near_t;
    return mint <= far_t && near_t <= maxt;
}

// Correctly rounded 1/x (what `1.0f / x` gives) in 3 instructions: the hardware estimate (within 1 ulp)
// and one FMA Newton step. Checked against the correctly rounded division for all 2^32 inputs on gfx950
// (tools/rcp_exhaustive.hip, tests/test_gpu_parity.py::test_fast_reciprocal_exhaustive): identical for
// |x| in [2^-125, 2^126); outside that range the caller must use the division.
NHD float rcp_rn(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
// 1/det of Mesh::rayIntersect: every det the test does not reject (|det| >= 1e-8 or NaN) takes rcp_rn
// unless it is >= 2^126 in magnitude (then the division); rejected dets may get any value
NHD float tri_inv_det(float det) {
    float r = rcp_rn(det);
    if (__builtin_expect(fabsf(det) >= 0x1p126f, 0)) r = 1.0f / det;
    return r;
}

// Mesh::rayIntersect (mesh.cpp:101-139): edges from the vertices, as the reference computes them
NHD bool tri_test(float4 a, float4 b, float4 c, F3 o, F3 d, float mint, float maxt, float &t, float &u, float &v) {
    const F3 p0 = f3(a.x, a.y, a.z), e1 = sub(f3(b.x, b.y, b.z), p0), e2 = sub(f3(c.x, c.y, c.z), p0);
    F3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    if (det > -1e-8f && det < 1e-8f) return false;
    float inv_det = tri_inv_det(det);
    F3 tvec = sub(o, p0);
    u = dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return false;
    F3 qvec = cross(tvec, e1);
    v = dot(d, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(e2, qvec) * inv_det;
    return t >= mint && t <= maxt;
}

// Two Moller-Trumbore tests at once, one per component of packed-FP32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: each component is the IEEE single-precision result of the same operation, so the
// pair computes exactly what two tri_test_nb calls compute, in half the VALU issue slots). Returns
// the hit predicates without the maxt bound (t_ok: t >= mint; the caller applies t <= maxt in
// primitive order, since a hit of the first shrinks maxt for the second).
typedef float f2 __attribute__((ext_vector_type(2)));
struct P3 {
    f2 x, y, z;
};
NHD P3 psub(P3 a, P3 b) { return P3{a.x - b.x, a.y - b.y, a.z - b.z}; }
NHD P3 pcross(P3 a, P3 b) { return P3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
NHD f2 pdot(P3 a, P3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
// the pair test from the vertex p0 and the edges e1 = p1 - p0, e2 = p2 - p0 (mesh.cpp:105-106), which the LDS pair
// records of small scenes hold precomputed (the same IEEE subtractions, done once when the records are staged)
NHD void tri_test_pair_e(const P3 &p0, const P3 &e1, const P3 &e2, F3 o, F3 d, float mint, f2 &t, f2 &u, f2 &v,
                         bool &ok0, bool &ok1) {
    const P3 po{f2{o.x, o.x}, f2{o.y, o.y}, f2{o.z, o.z}}, pd{f2{d.x, d.x}, f2{d.y, d.y}, f2{d.z, d.z}};
    const P3 pvec = pcross(pd, e2);
    const f2 det = pdot(e1, pvec);
    const f2 inv_det = f2{tri_inv_det(det.x), tri_inv_det(det.y)};
    const P3 tvec = psub(po, p0);
    u = pdot(tvec, pvec) * inv_det;
    const P3 qvec = pcross(tvec, e1);
    v = pdot(pd, qvec) * inv_det;
    t = pdot(e2, qvec) * inv_det;
    const f2 uv = u + v;
    ok0 = !(det.x > -1e-8f && det.x < 1e-8f) & !(u.x < 0.0f || u.x > 1.0f) & !(v.x < 0.0f || uv.x > 1.0f) &
          (t.x >= mint);
    ok1 = !(det.y > -1e-8f && det.y < 1e-8f) & !(u.y < 0.0f || u.y > 1.0f) & !(v.y < 0.0f || uv.y > 1.0f) &
          (t.y >= mint);
}
NHD void tri_test_pair_p(const P3 &p0, const P3 &p1, const P3 &p2, F3 o, F3 d, float mint, f2 &t, f2 &u, f2 &v,
                         bool &ok0, bool &ok1) {
    tri_test_pair_e(p0, psub(p1, p0), psub(p2, p0), o, d, mint, t, u, v, ok0, ok1);
}
NHD void tri_test_pair(float4 a0, float4 b0, float4 c0, float4 a1, float4 b1, float4 c1, F3 o, F3 d, float mint,
                       f2 &t, f2 &u, f2 &v, bool &ok0, bool &ok1) {
    const P3 p0{f2{a0.x, a1.x}, f2{a0.y, a1.y}, f2{a0.z, a1.z}};
    const P3 p1{f2{b0.x, b1.x}, f2{b0.y, b1.y}, f2{b0.z, b1.z}};
    const P3 p2{f2{c0.x, c1.x}, f2{c0.y, c1.y}, f2{c0.z, c1.z}};
    tri_test_pair_p(p0, p1, p2, o, d, mint, t, u, v, ok0, ok1);
}

// tri_test without early exits: the same predicates on the same values (so the same answer, NaNs
// included), evaluated in full. In SIMT code an early return only skips work when every lane of
// the wave takes it; otherwise it costs a branch and exec-mask bookkeeping per test.
NHD bool tri_test_nb(float4 a, float4 b, float4 c, F3 o, F3 d, float mint, float maxt, float &t, float &u, float &v) {
    const F3 p0 = f3(a.x, a.y, a.z), e1 = sub(f3(b.x, b.y, b.z), p0), e2 = sub(f3(c.x, c.y, c.z), p0);
    const F3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    const float inv_det = tri_inv_det(det);
    const F3 tvec = sub(o, p0);
    u = dot(tvec, pvec) * inv_det;
    const F3 qvec = cross(tvec, e1);
    v = dot(d, qvec) * inv_det;
    t = dot(e2, qvec) * inv_det;
    const bool ok_det = !(det > -1e-8f && det < 1e-8f);
    const bool ok_u = !(u < 0.0f || u > 1.0f);
    const bool ok_v = !(v < 0.0f || u + v > 1.0f);
    return ok_det & ok_u & ok_v & (t >= mint) & (t <= maxt);
}

// box_test for rays whose 1/d components are all finite (no zero direction component): the
// reference's per-axis t1/t2 swap is min/max (the products are monotone in the bounds, and no NaN
// arises: finite differences times finite r), and its running max/min with the per-axis early-outs
// give the same final near/far as one max/min over the axes. Returns the hit test; near in near_out.
NHD bool box_test_finite(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, F3 o, F3 r, float mint,
                         float maxt, float &near_out) {
    const float ax = (mnx - o.x) * r.x, bx = (mxx - o.x) * r.x;
    const float ay = (mny - o.y) * r.y, by = (mxy - o.y) * r.y;
    const float az = (mnz - o.z) * r.z, bz = (mxz - o.z) * r.z;
    const float near_t = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float far_t = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    near_out = near_t;
    return (near_t <= far_t) & (mint <= far_t) & (near_t <= maxt);
}

// box_test_finite for two boxes at once: the slab products in packed FP32 (component i = box i, the
// same IEEE operations), the min / max reductions per box as box_test_finite does them
NHD void box_test_finite_pair(f2 mnx, f2 mny, f2 mnz, f2 mxx, f2 mxy, f2 mxz, float o_x, float o_y, float o_z,
                              float r_x, float r_y, float r_z, float mint, float maxt, bool &hit0, bool &hit1,
                              float &near0, float &near1) {
    const f2 ox{o_x, o_x}, oy{o_y, o_y}, oz{o_z, o_z}, rx{r_x, r_x}, ry{r_y, r_y}, rz{r_z, r_z};
    const f2 ax = (mnx - ox) * rx, bx = (mxx - ox) * rx;
    const f2 ay = (mny - oy) * ry, by = (mxy - oy) * ry;
    const f2 az = (mnz - oz) * rz, bz = (mxz - oz) * rz;
    const float n0 = fmaxf(fmaxf(fminf(ax.x, bx.x), fminf(ay.x, by.x)), fminf(az.x, bz.x));
    const float f0 = fminf(fminf(fmaxf(ax.x, bx.x), fmaxf(ay.x, by.x)), fmaxf(az.x, bz.x));
    const float n1 = fmaxf(fmaxf(fminf(ax.y, bx.y), fminf(ay.y, by.y)), fminf(az.y, bz.y));
    const float f1 = fminf(fminf(fmaxf(ax.y, bx.y), fmaxf(ay.y, by.y)), fmaxf(az.y, bz.y));
    near0 = n0;
    near1 = n1;
    hit0 = (n0 <= f0) & (mint <= f0) & (n0 <= maxt);
    hit1 = (n1 <= f1) & (mint <= f1) & (n1 <= maxt);
}

// Sphere::rayIntersect (sphere.cpp:67-94)
NHD bool sphere_test(float4 a, F3 o, F3 d, float mint, float maxt, float &t) {
    F3 L = sub(o, f3(a.x, a.y, a.z));
    float qa = dot(d, d);
    float qb = 2.f * dot(d, L);
    float qc = dot(L, L) - a.w * a.w;
    float discr = qb * qb - 4.f * qa * qc;
    if (discr < 0.f) return false;
    const float tmin = (-qb - f_sqrt(discr)) / 2 / qa;
    const float tmax = (-qb + f_sqrt(discr)) / 2 / qa;
    if (mint <= tmin && maxt >= tmin) { t = tmin; return true; }
    if (mint <= tmax && maxt >= tmax) { t = tmax; return true; }
    return false;
}

struct Traversal {
    const float4 *nodes;
    const int2 *leaves;
    const float4 *prims;
    const float4 *wnodes;  // 4-wide collapse of the same tree (kWideF4 float4 per node), see Tracer4
    // LDS-staged scenes (wf_bounce): records k and k+1 interleaved component by component, kPairF4 float4
    // per k, so a primitive pair loads straight into packed-FP32 register pairs (leaf_test<.., PAIRS>)
    const float4 *ppairs;
    // LDS-staged scenes: each triangle's shading frame when its mesh has no normals (Mesh::setHitInformation's
    // Frame(normalized(cross(p1 - p0, p2 - p0))), mesh.cpp:180-190), 3 float4 (s, t, n) per record, computed at
    // staging by the same arithmetic; nullptr: hit_info computes it
    const float4 *frames;
    // the first n_top wide nodes are the top of the tree (the nodes most rays visit, nh_api.hip numbers
    // them first); the persistent traversal kernels read those from an LDS copy
    int n_top;
};
// pair k: (a.x a.x') (a.y a.y') | (a.z a.z') (a.w a.w') | (e1.x e1.x') (e1.y e1.y') | (e1.z e1.z') (e2.x e2.x') |
//         (e2.y e2.y') (e2.z e2.z') | (c.w c.w') (0 0)   -- unprimed record k, primed record k+1; a = p0 (a sphere's
//         centre and radius), e1 = p1 - p0, e2 = p2 - p0 (triangles only)
constexpr int kPairF4 = 6;

// primitive record type / leaf-end bits (word 2 .w of the record), and the BSDF type of the owning
// shape in bits 2-3 (the material key of the sorted shade queues)
constexpr int kPrimSphere = 1, kPrimLeafEnd = 2, kPrimMatShift = 2;
// an isolated sphere (record 2 .w bit; record 1 .x holds the host's margin m): see trace_next
constexpr int kPrimIsolated = 16;
NHD bool prim_is_tri(float4 c) { return (__float_as_int(c.w) & kPrimSphere) == 0; }
NHD int prim_material(float4 c) { return (__float_as_int(c.w) >> kPrimMatShift) & 3; }

// Test the primitives of one leaf. Returns true when an any-hit query is answered.
template <bool ANY, bool STATS, bool PAIRS = false>
NHD bool leaf_test(const Traversal &tv, int leaf, F3 o, F3 d, float mint, float &maxt, Hit &best, bool &found,
                   TravStats &st) {
    const int2 lf = tv.leaves[leaf];
    if constexpr (PAIRS) {  // interleaved pair records: no AoS -> pair shuffles
        for (int k = lf.x, e = lf.x + lf.y; k < e; k += 2) {
            const float4 *pp = tv.ppairs + (size_t)kPairF4 * k;
            const float4 q0 = pp[0], q1 = pp[1], q2 = pp[2], q3 = pp[3], q4 = pp[4], q5 = pp[5];
            const P3 p0{f2{q0.x, q0.y}, f2{q0.z, q0.w}, f2{q1.x, q1.y}};
            const P3 e1{f2{q2.x, q2.y}, f2{q2.z, q2.w}, f2{q3.x, q3.y}};
            const P3 e2{f2{q3.z, q3.w}, f2{q4.x, q4.y}, f2{q4.z, q4.w}};
            f2 pt, pu, pv;
            bool ok0, ok1;
            tri_test_pair_e(p0, e1, e2, o, d, mint, pt, pu, pv, ok0, ok1);
            const bool has1 = k + 1 < e;
            if (!STATS && !((__float_as_int(q5.x) | (has1 ? __float_as_int(q5.y) : 0)) & kPrimSphere)) {
                // two triangles (or the leaf's last one): the loop below's acceptance in primitive order, as selects
                // (a hit needs t <= the running maxt; it replaces the best on t < maxt or a later record)
                if (ANY) {
                    if ((ok0 && pt.x <= maxt) || (has1 && ok1 && pt.y <= maxt)) return true;
                    continue;
                }
                const bool h0 = ok0 && pt.x <= maxt;
                const bool u0 = h0 && (pt.x < maxt || k > best.k);
                maxt = u0 ? pt.x : maxt;
                best.t = u0 ? pt.x : best.t;
                best.u = u0 ? pu.x : best.u;
                best.v = u0 ? pv.x : best.v;
                best.k = u0 ? k : best.k;
                const bool h1 = has1 && ok1 && pt.y <= maxt;
                const bool u1 = h1 && (pt.y < maxt || k + 1 > best.k);
                maxt = u1 ? pt.y : maxt;
                best.t = u1 ? pt.y : best.t;
                best.u = u1 ? pu.y : best.u;
                best.v = u1 ? pv.y : best.v;
                best.k = u1 ? k + 1 : best.k;
                found = found || u0 || u1;
                continue;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j == 1 && k + 1 >= e) break;
                if (STATS) st.prims++;
                float t = j ? pt.y : pt.x, u = j ? pu.y : pu.x, v = j ? pv.y : pv.x;
                const float cw = j ? q5.y : q5.x;
                bool hit;
                if ((__float_as_int(cw) & kPrimSphere) == 0) {
                    hit = (j ? ok1 : ok0) && t <= maxt;
                } else {
                    u = v = 0.f;
                    const float4 a = j ? make_float4(q0.y, q0.w, q1.y, q1.w) : make_float4(q0.x, q0.z, q1.x, q1.z);
                    hit = sphere_test(a, o, d, mint, maxt, t);
                }
                if (!hit) continue;
                if (ANY) return true;
                if (t < maxt || k + j > best.k) {
                    found = true;
                    maxt = t;
                    best.t = t;
                    best.u = u;
                    best.v = v;
                    best.k = k + j;
                }
            }
        }
        return false;
    }
    // primitives in pairs: both triangle tests in packed FP32 (tri_test_pair), then accepted in
    // order -- a hit of the first shrinks maxt before the second is bounded by it
    for (int k = lf.x, e = lf.x + lf.y; k < e; k += 2) {
        const int k1 = k + 1 < e ? k + 1 : k;
        const float4 a0 = tv.prims[3 * k], b0 = tv.prims[3 * k + 1], c0 = tv.prims[3 * k + 2];
        const float4 a1 = tv.prims[3 * k1], b1 = tv.prims[3 * k1 + 1], c1 = tv.prims[3 * k1 + 2];
        f2 pt, pu, pv;
        bool ok0, ok1;
        tri_test_pair(a0, b0, c0, a1, b1, c1, o, d, mint, pt, pu, pv, ok0, ok1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j == 1 && k1 == k) break;
            const float4 &a = j ? a1 : a0, &c = j ? c1 : c0;
            if (STATS) st.prims++;
            float t = j ? pt.y : pt.x, u = j ? pu.y : pu.x, v = j ? pv.y : pv.x;
            bool hit;
            if (prim_is_tri(c)) {
                hit = (j ? ok1 : ok0) && t <= maxt;
            } else {
                u = v = 0.f;
                hit = sphere_test(a, o, d, mint, maxt, t);
            }
            if (!hit) continue;
            if (ANY) return true;
            if (t < maxt || k + j > best.k) {
                found = true;
                maxt = t;
                best.t = t;
                best.u = u;
                best.v = v;
                best.k = k + j;
            }
        }
    }
    return false;
}

// The primitives of one leaf tested by a G-lane group that carries one ray (every lane the same ray, the same
// traversal): lane j of the group tests primitive start + j (+ G, + 2G for longer leaves), each against the maxt at
// the leaf's entry, and the group reduces the accepted hits to the smallest t, ties to the largest leaf position k.
// That is the sequential loop's answer: it accepts each primitive whose t <= the running maxt, so its last accepted
// primitive is the latest one of the leaf's minimum t; a candidate above that minimum never wins either way (a
// sphere's candidate t does not depend on maxt: tmin if it is past mint, else tmax). The update across leaves is the
// sequential one (t < maxt, or a later primitive on a tie). Any hit: the group's OR. Counters match the sequential
// loop's (every primitive of the leaf; an any-hit query up to its first hit).
template <bool ANY, bool STATS, int G>
NHD bool leaf_test_coop(const Traversal &tv, int leaf, F3 o, F3 d, float mint, float &maxt, Hit &best, bool &found,
                        TravStats &st) {
    const int lane = threadIdx.x & 63, gl = lane & (G - 1), gbase = lane & ~(G - 1);
    const int2 lf = tv.leaves[leaf];
    for (int base = lf.x, e = lf.x + lf.y; base < e; base += G) {
        const int k = base + gl;
        bool acc = false;
        float t = INFINITY, u = 0.f, v = 0.f;
        if (k < e) {
            const float4 a = tv.prims[3 * k], b = tv.prims[3 * k + 1], c = tv.prims[3 * k + 2];
            if (prim_is_tri(c)) acc = tri_test_nb(a, b, c, o, d, mint, maxt, t, u, v);
            else acc = sphere_test(a, o, d, mint, maxt, t);
        }
        const unsigned long long grp = (__ballot(acc) >> gbase) & ((1ull << G) - 1ull);
        if (ANY) {
            if (grp) {
                if (STATS && gl == 0) st.prims += (uint32_t)(__ffsll((long long)grp));  // up to the first hit
                return true;
            }
            if (STATS && gl == 0) st.prims += (uint32_t)min(G, e - base);
            continue;
        }
        if (STATS && gl == 0) st.prims += (uint32_t)min(G, e - base);
        if (!grp) continue;
        float rt = acc ? t : INFINITY;
        int rk = acc ? k : -1;
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) {
            const float ot = __shfl_xor(rt, off, G);
            const int ok = __shfl_xor(rk, off, G);
            if (ok >= 0 && (rk < 0 || ot < rt || (ot == rt && ok > rk))) {
                rt = ot;
                rk = ok;
            }
        }
        const float wu = __shfl(u, rk - base, G), wv = __shfl(v, rk - base, G);
        if (rt < maxt || rk > best.k) {
            found = true;
            maxt = rt;
            best.t = rt;
            best.u = wu;
            best.v = wv;
            best.k = rk;
        }
    }
    return false;
}

template <bool ANY, bool STATS, bool PAIRS, int G>
NHD bool leaf_any(const Traversal &tv, int leaf, F3 o, F3 d, float mint, float &maxt, Hit &best, bool &found,
                  TravStats &st) {
    if constexpr (G > 1) return leaf_test_coop<ANY, STATS, G>(tv, leaf, o, d, mint, maxt, best, found, st);
    else return leaf_test<ANY, STATS, PAIRS>(tv, leaf, o, d, mint, maxt, best, found, st);
}

// Inner-node fields read as scalars straight from the node record (float i of node n: nf[i], nf = the node's first
// float): [0..5] the left child's box (min xyz, max xyz), [6..11] the right child's, int [12] / [13] their refs. The
// float4 form (n0, n1, n2) let the compiler pick a child's six bounds by selecting between addresses of local float4
// copies, which put those copies in scratch memory: a scratch store and reload in every node visit of every traversal.
NHD const float *node_f(const Traversal &tv, int n) { return reinterpret_cast<const float *>(tv.nodes + 4 * n); }
NHD int node_ref(const float *nf, int side) { return reinterpret_cast<const int *>(nf)[12 + side]; }

// Child box of an inner node: side 0 = left, 1 = right (its six bounds read from the record at nf + 6 side). fin:
// every 1/d component is finite (box_test_finite applies)
NHD bool child_box_test(const float *nf, int side, F3 o, F3 d, F3 r, float mint, float maxt, float &near_t, bool fin) {
    const float *c = nf + 6 * side;
    const float mnx = c[0], mny = c[1], mnz = c[2], mxx = c[3], mxy = c[4], mxz = c[5];
    if (fin) return box_test_finite(mnx, mny, mnz, mxx, mxy, mxz, o, r, mint, maxt, near_t);
    return box_test(mnx, mny, mnz, mxx, mxy, mxz, o, d, r, mint, maxt, near_t);
}

// Both child boxes of an inner node; rays with all 1/d finite take the branch-free packed slab test (box_test_finite:
// the same answers as the reference's branchy form for them), the others the reference's form
NHD void node_box_tests(const float *nf, F3 o, F3 d, F3 r, float mint, float maxt, bool fin, bool &hl, bool &hr,
                        float &nl, float &nr) {
    const float l0 = nf[0], l1 = nf[1], l2 = nf[2], l3 = nf[3], l4 = nf[4], l5 = nf[5];
    const float r0 = nf[6], r1 = nf[7], r2 = nf[8], r3 = nf[9], r4 = nf[10], r5 = nf[11];
    if (fin) {
        box_test_finite_pair(f2{l0, r0}, f2{l1, r1}, f2{l2, r2}, f2{l3, r3}, f2{l4, r4}, f2{l5, r5}, o.x, o.y, o.z, r.x,
                             r.y, r.z, mint, maxt, hl, hr, nl, nr);
    } else {
        hl = box_test(l0, l1, l2, l3, l4, l5, o, d, r, mint, maxt, nl);
        hr = box_test(r0, r1, r2, r3, r4, r5, o, d, r, mint, maxt, nr);
    }
}

// Closest / any hit. stk points at this thread's first LDS stack slot; consecutive
// entries are `stride` words apart (lane-interleaved, bank-conflict free). An entry is
// (parent inner node << 1) | side: the deferred child's box is tested again when it is
// popped, with the maxt of that moment -- the reference's visit-time test verbatim.
// G > 1: the ray is carried by a G-lane group (leaf primitives tested cooperatively, leaf_test_coop).
template <int DEPTH, bool ORDERED, bool ANY, bool STATS, bool PAIRS = false, int G = 1>
NHD bool trace(const Traversal &tv, const DScene &S, F3 o, F3 d, float mint, float maxt, Hit &best, uint32_t *stk,
               int stride, TravStats &st) {
    // adaptive ray epsilon (bvh.cpp:407-410)
    if (mint == kEps) mint = e_max(mint, mint * e_max(fabsf(o.x), e_max(fabsf(o.y), fabsf(o.z))));
    // counters: one lane of a group carrying the ray counts for it
    const bool lead = G == 1 || (threadIdx.x & (G - 1)) == 0;
    best.k = -1;
    best.t = INFINITY;
    if (S.root_kind == 0 || maxt < mint) return false;
    const F3 r = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const bool fin = isfinite(r.x) & isfinite(r.y) & isfinite(r.z);
    bool found = false;
    float near_t;
    if (STATS && lead) st.boxes++;
    if (fin ? !box_test_finite(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1],
                               S.root_max[2], o, r, mint, maxt, near_t)
            : !box_test(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1], S.root_max[2], o,
                        d, r, mint, maxt, near_t))
        return false;
    if (S.root_kind == 2) {
        bool any = leaf_any<ANY, STATS, PAIRS, G>(tv, 0, o, d, mint, maxt, best, found, st);
        return ANY ? any : found;
    }
    int sp = 0;
    int cur = 0;
    for (;;) {
        while (cur >= 0) {
            const float *nf = node_f(tv, cur);
            const int ref_l = node_ref(nf, 0), ref_r = node_ref(nf, 1);
            if (STATS && lead) { st.nodes++; st.boxes += 2; }
            float nl, nr;
            bool hl, hr;
            node_box_tests(nf, o, d, r, mint, maxt, fin, hl, hr, nl, nr);
            int next;
            if (hl && hr) {
                const bool right_first = ORDERED && nr < nl;
                stk[sp * stride] = ((uint32_t)cur << 1) | (right_first ? 0u : 1u);
                ++sp;
                next = right_first ? ref_r : ref_l;
            } else if (hl) {
                next = ref_l;
            } else if (hr) {
                next = ref_r;
            } else {
                break;
            }
            if (next >= 0) {
                cur = next;
                continue;
            }
            if (leaf_any<ANY, STATS, PAIRS, G>(tv, ~next, o, d, mint, maxt, best, found, st)) return true;
            break;
        }
        // pop: re-test the deferred child against the current maxt
        cur = -1;
        while (sp > 0) {
            --sp;
            const uint32_t e = stk[sp * stride];
            const int parent = (int)(e >> 1), side = (int)(e & 1u);
            const float *nf = node_f(tv, parent);
            if (STATS && lead) st.boxes++;
            if (!child_box_test(nf, side, o, d, r, mint, maxt, near_t, fin)) continue;
            const int ref = node_ref(nf, side);
            if (ref >= 0) {
                cur = ref;
                break;
            }
            if (leaf_any<ANY, STATS, PAIRS, G>(tv, ~ref, o, d, mint, maxt, best, found, st)) return true;
        }
        if (cur < 0) break;
    }
    (void)DEPTH;
    return ANY ? false : found;
}

// The closest hit of a path's next ray, which leaves the surface of primitive k_prev (-1: none). When k_prev is an
// isolated sphere -- the host found its box, grown by 2m, apart from every other primitive's box -- and the ray
// starts within m of that box and meets the sphere at t >= 2 mint, the traversal's answer is that sphere at that t,
// so the tree is not walked. Why: every primitive a traversal accepts at t lies (up to rounding far below m) at
// o + t d inside its own box; on [mint, t] the ray stays inside the sphere's box grown by m (both ends are in that
// convex box), which no other primitive's box reaches, so no other primitive is accepted at or before t and the
// answer -- the smallest accepted t, ties to the later record -- is the sphere's, found with the maxt any order of
// visits tests it with (>= t). No box on the way culls it: each holds the sphere's box, the ray's exit from it is
// past t (up to rounding) >= 2 mint, and the entry before the exit. The sphere test is sphere_test, with the
// traversal's adaptive mint. Counted as one primitive test (no node or box).
template <bool STATS, int G = 1>
NHD bool iso_sphere_hit(const Traversal &tv, int k_prev, F3 o, F3 d, float mint, float maxt, Hit &best,
                        TravStats &st) {
    if (k_prev < 0) return false;
    const float4 c = tv.prims[3 * k_prev + 2];
    if (!(__float_as_int(c.w) & kPrimIsolated)) return false;
    if (mint == kEps) mint = e_max(mint, mint * e_max(fabsf(o.x), e_max(fabsf(o.y), fabsf(o.z))));  // as trace
    if (maxt < mint) return false;
    const float4 a = tv.prims[3 * k_prev];
    const float lim = a.w + tv.prims[3 * k_prev + 1].x;
    if (!(fabsf(o.x - a.x) <= lim && fabsf(o.y - a.y) <= lim && fabsf(o.z - a.z) <= lim)) return false;
    float t;
    if (!sphere_test(a, o, d, mint, maxt, t) || !(t >= 2.f * mint)) return false;
    best.t = t;
    best.u = 0.f;
    best.v = 0.f;
    best.k = k_prev;
    if (STATS && (G == 1 || (threadIdx.x & (G - 1)) == 0)) st.prims++;
    return true;
}

// trace (closest hit) of a path's next ray from the surface of primitive k_prev, with the isolated-sphere answer
template <int DEPTH, bool ORDERED, bool STATS, bool PAIRS = false, int G = 1, bool ISO = true>
NHD bool trace_next(const Traversal &tv, const DScene &S, int k_prev, F3 o, F3 d, float mint, float maxt, Hit &best,
                    uint32_t *stk, int stride, TravStats &st) {
#ifndef NH_AB_NO_ISO  // cost attribution builds only: the isolated-sphere test compiled out
    if (ISO && S.iso_spheres && S.root_kind != 0 && iso_sphere_hit<STATS, G>(tv, k_prev, o, d, mint, maxt, best, st))
        return true;
#endif
    return trace<DEPTH, ORDERED, false, STATS, PAIRS, G>(tv, S, o, d, mint, maxt, best, stk, stride, st);
}



// Traversal stack of one lane for the persistent kernels: the top K entries live in LDS
// (lane-interleaved, `stride` words apart), deeper entries spill to the lane's own region of a
// global buffer. LDS per lane no longer scales with the tree depth, so deep trees (the 10M-triangle
// C5 scene needs 35 entries) keep the occupancy that registers allow.
template <int K>
struct RingStack {
    static_assert((K & (K - 1)) == 0, "K must be a power of two");
    uint32_t *lds;   // this lane's first LDS slot
    int stride;
    uint32_t *glob;  // this lane's spill area (max depth - K entries)
    NHD void push(int i, uint32_t e) {  // i = index of the new entry
        uint32_t *slot = lds + (i & (K - 1)) * stride;
        if (i >= K) glob[i - K] = *slot;  // the slot holds entry i - K: spill it
        *slot = e;
    }
    NHD uint32_t pop(int i) {  // i = index of the top entry
        uint32_t *slot = lds + (i & (K - 1)) * stride;
        const uint32_t e = *slot;
        if (i >= K) *slot = glob[i - K];  // entry i - K moves back into the window
        return e;
    }
};

// Resumable form of trace(): identical visits, box/primitive tests and order (hence identical
// results and counters), but one unit of work per step() -- one inner node, one primitive, or
// one stack pop -- so a persistent wave can hand finished lanes new rays between steps instead
// of idling until its slowest lane is done (nh_wavefront.hip wf_trace_pt).
template <bool ORDERED, bool ANY, bool STATS, class Stack>
struct Tracer {
    F3 o, d, r;
    float mint, maxt;
    int cur;      // inner node to visit next, or -1
    int k, kend;  // primitive range of the leaf under test
    int sp;
    bool found, done;
    bool fin;  // every 1/d component finite: branch-free slab tests (box_test_finite)
    Hit best;

    NHD void begin(const DScene &S, const Traversal &tv, F3 o_, F3 d_, float mint_, float maxt_, TravStats &st) {
        o = o_;
        d = d_;
        mint = mint_;
        maxt = maxt_;
        // adaptive ray epsilon (bvh.cpp:407-410)
        if (mint == kEps) mint = e_max(mint, mint * e_max(fabsf(o.x), e_max(fabsf(o.y), fabsf(o.z))));
        best.k = -1;
        best.t = INFINITY;
        found = false;
        done = true;
        sp = 0;
        cur = -1;
        k = kend = 0;
        if (S.root_kind == 0 || maxt < mint) return;
        r = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        fin = isfinite(r.x) & isfinite(r.y) & isfinite(r.z);
        float near_t;
        if (STATS) st.boxes++;
        if (fin ? !box_test_finite(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1],
                                   S.root_max[2], o, r, mint, maxt, near_t)
                : !box_test(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1], S.root_max[2],
                            o, d, r, mint, maxt, near_t))
            return;
        done = false;
        if (S.root_kind == 2) {
            const int2 lf = tv.leaves[0];
            k = lf.x;
            kend = lf.x + lf.y;
        } else {
            cur = 0;
        }
    }

    NHD void step(const Traversal &tv, Stack &stk, TravStats &st) {
        if (k < kend) {  // one primitive of the current leaf
            const float4 a = tv.prims[3 * k], b = tv.prims[3 * k + 1], c = tv.prims[3 * k + 2];
            if (STATS) st.prims++;
            float t, u = 0.f, v = 0.f;
            const bool hit = prim_is_tri(c) ? tri_test(a, b, c, o, d, mint, maxt, t, u, v)
                                                        : sphere_test(a, o, d, mint, maxt, t);
            if (hit) {
                if (ANY) {
                    found = true;
                    done = true;
                    return;
                }
                if (t < maxt || k > best.k) {
                    found = true;
                    maxt = t;
                    best.t = t;
                    best.u = u;
                    best.v = v;
                    best.k = k;
                }
            }
            ++k;
            return;
        }
        if (cur >= 0) {  // one inner node: test both child boxes
            const float *nf = node_f(tv, cur);
            const int ref_l = node_ref(nf, 0), ref_r = node_ref(nf, 1);
            if (STATS) { st.nodes++; st.boxes += 2; }
            float nl, nr;
            bool hl, hr;
            node_box_tests(nf, o, d, r, mint, maxt, fin, hl, hr, nl, nr);
            int next;
            if (hl && hr) {
                const bool right_first = ORDERED && nr < nl;
                stk.push(sp, ((uint32_t)cur << 1) | (right_first ? 0u : 1u));
                ++sp;
                next = right_first ? ref_r : ref_l;
            } else if (hl) {
                next = ref_l;
            } else if (hr) {
                next = ref_r;
            } else {
                cur = -1;
                return;
            }
            enter(tv, next);
            return;
        }
        if (sp > 0) {  // one deferred child: re-test its box against the current maxt
            --sp;
            const uint32_t e = stk.pop(sp);
            const int parent = (int)(e >> 1), side = (int)(e & 1u);
            const float *nf = node_f(tv, parent);
            if (STATS) st.boxes++;
            float near_t;
            if (!child_box_test(nf, side, o, d, r, mint, maxt, near_t, fin)) return;
            enter(tv, node_ref(nf, side));
            return;
        }
        done = true;
    }

    NHD void enter(const Traversal &tv, int ref) {
        if (ref >= 0) {
            cur = ref;
        } else {
            const int2 lf = tv.leaves[~ref];
            k = lf.x;
            kend = lf.x + lf.y;
            cur = -1;
        }
    }
};

// ---------------------------------------------------------------------------------------------
// 4-wide traversal of the same tree. nh_api.hip collapses the reference's binary tree: a wide
// node's children are binary descendants (an inner child is replaced by its two children, the
// largest-area one first, until there are 4), in left-first DFS order, with the descendants'
// own boxes -- no new boxes. Skipping the boxes of the collapsed intermediate nodes changes no
// result: a descendant's box lies inside its ancestor's (the reference builds every box as the
// union of its primitives), and the slab arithmetic is monotone in the bounds, so the rounded
// [near, far] of a descendant lies inside its ancestor's -- whenever the descendant passes
// `mint <= far && near <= maxt`, the skipped ancestor would have passed too (with the same or a
// larger maxt, since maxt only shrinks). Leaves are primitive ranges ending at the record whose
// kPrimLeafEnd bit is set (no leaf-table fetch).
//
// Wide node (128 B, one cache line) = 8 x float4:
//   [0..5] min.x[4], min.y[4], min.z[4], max.x[4], max.y[4], max.z[4] of the 4 child slots
//   [6]    int4 child refs: >= 0 wide node, kWideEmpty unused slot, else leaf ~first primitive
//   [7]    unused
constexpr int kWideF4 = 8;
// work per Tracer4::step for a lane: up to this many wide nodes, then up to two primitives
#ifndef NH_NODES_PER_STEP
#define NH_NODES_PER_STEP 1
#endif

constexpr int kWideEmpty = (int)0x80000000;
// the two primitive records of a step tested as a packed pair (tri_test_pair) or one after the other
#ifndef NH_WIDE_PAIR
#define NH_WIDE_PAIR 1
#endif
// the four child boxes of a wide node tested as two packed pairs (box_test_finite_pair): off, the
// extra live registers spill at 5 waves/SIMD (bumpy-1M 1260 vs 1404 Msamples/s)
#ifndef NH_WIDE_PACKED_BOX
#define NH_WIDE_PACKED_BOX 0
#endif

// Traversal stack of one lane, (ref, entry distance) pairs: the top K entries live in LDS
// (lane-interleaved, `stride` words apart), deeper entries spill to a global area, lane-interleaved too: spill entry
// j of lane g at glob[j * lanes + g] (glob and lanes uniform). The lane keeps only its 32-bit index g live -- a
// per-lane 64-bit pointer into its own region was two more VGPRs, which the persistent kernels spilled to scratch at
// their 96-VGPR budget -- and lanes that spill at the same depth write neighbouring words.
template <int K>
struct RingStack2 {
    static_assert((K & (K - 1)) == 0, "K must be a power of two");
    int *lds_ref;      // this lane's first LDS slot (refs)
    float *lds_near;   // this lane's first LDS slot (entry distances)
    int stride;
    int2 *glob;        // spill area (uniform)
    unsigned lanes;    // lanes sharing it (uniform)
    unsigned g;        // this lane's index
    NHD int2 &spill(int j) const { return glob[(size_t)(unsigned)j * lanes + g]; }
    NHD void push(int i, int ref, float nr) {
        const int o = (i & (K - 1)) * stride;
        if (i >= K) spill(i - K) = make_int2(lds_ref[o], __float_as_int(lds_near[o]));
        lds_ref[o] = ref;
        lds_near[o] = nr;
    }
    // entries i0 .. i0+m-1 (m <= M < K; M = 3 for 4-wide nodes, 7 for 8-wide ones) are about to be written with
    // put(): spill the entries K below them that still occupy their ring slots
    template <int M = 3>
    NHD void reserve(int i0, int m) {
        static_assert(M < K, "a node's deferred children must fit the LDS window");
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int i = i0 + j;
            if (j < m && i >= K) {
                const int o = (i & (K - 1)) * stride;
                spill(i - K) = make_int2(lds_ref[o], __float_as_int(lds_near[o]));
            }
        }
    }
    NHD void put(int i, int ref, float nr) {
        const int o = (i & (K - 1)) * stride;
        lds_ref[o] = ref;
        lds_near[o] = nr;
    }
    NHD void pop(int i, int &ref, float &nr) {
        const int o = (i & (K - 1)) * stride;
        ref = lds_ref[o];
        nr = lds_near[o];
        if (i >= K) {
            const int2 e = spill(i - K);
            lds_ref[o] = e.x;
            lds_near[o] = __int_as_float(e.y);
        }
    }
};

// ORDERED: nearer first, equal distances in slot (= left-first DFS) order; REFERENCE: slot order
template <bool ORDERED>
NHD bool wide_before(bool va, float na, int sa, bool vb, float nb, int sb) {
    if (!va) return false;
    if (!vb) return true;
    if (ORDERED && na != nb) return na < nb;
    return sa < sb;
}

// wide_before for slots a < b as a branch-free 0/1: does child a come before child b?
template <bool ORDERED>
NHD int wide_first(bool va, float na, bool vb, float nb) {
    // valid before invalid; among valid: nearer first, equal near (never NaN for a hit) in slot order
    return (va & (!vb | !ORDERED | (na <= nb))) ? 1 : 0;
}

// Resumable 4-wide traversal (same step protocol as Tracer: one wide node, one primitive or one
// stack pop per step). Answers: smallest t, ties to the largest leaf-order position k.
// RT: the query kind is a run-time property of the lane (any_q, set before begin()), so one persistent launch
// serves closest-hit and any-hit rays together (wf_trace_pt2); otherwise ANY fixes it.
template <bool ORDERED, bool ANY, bool STATS, class Stack, bool RT = false>
struct Tracer4 {
    F3 o, d, r;
    float mint, maxt;
    int cur;  // wide node to visit next, or -1
    int k;    // primitive under test, or -1
    int sp;
    bool found, done;
    bool finite_r;  // all 1/d components finite: branch-free box tests (box_test_finite)
    bool any_q;     // RT: this lane's query is an any-hit query
    Hit best;

    NHD bool is_any() const { return RT ? any_q : ANY; }

    NHD void begin(const DScene &S, const Traversal &tv, F3 o_, F3 d_, float mint_, float maxt_, TravStats &st) {
        o = o_;
        d = d_;
        mint = mint_;
        maxt = maxt_;
        // adaptive ray epsilon (bvh.cpp:407-410)
        if (mint == kEps) mint = e_max(mint, mint * e_max(fabsf(o.x), e_max(fabsf(o.y), fabsf(o.z))));
        best.k = -1;
        best.t = INFINITY;
        found = false;
        done = true;
        sp = 0;
        cur = -1;
        k = -1;
        if (S.root_kind == 0 || maxt < mint) return;
        r = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        finite_r = fabsf(r.x) < INFINITY && fabsf(r.y) < INFINITY && fabsf(r.z) < INFINITY;
        float near_t;
        if (STATS) st.boxes++;
        if (!box_test(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1], S.root_max[2], o, d,
                      r, mint, maxt, near_t))
            return;
        done = false;
        if (S.root_kind == 2) k = tv.leaves[0].x;  // a single leaf: records up to the leaf-end bit
        else cur = 0;
    }

    // One iteration: (pop deferred children until one passes) -> (one wide node) -> (one primitive),
    // each part only if the lane has that work. A wave executes every part some lane needs anyway,
    // so chaining them lets a lane do a pop, a node and a primitive for the cost of one divergent
    // iteration; the per-lane sequence of operations (and so every result and counter) is unchanged.
    NHD void step(const Traversal &tv, Stack &stk, TravStats &st) { step(tv, stk, st, nullptr, 0); }
    // top / n_top: an LDS copy of the first n_top wide nodes (0: every node from tv.wnodes)
    NHD void step(const Traversal &tv, Stack &stk, TravStats &st, const float4 *top, int n_top) {
        if (k < 0 && cur < 0) {  // deferred children: the visit-time test against the current maxt
            while (sp > 0) {
                int ref;
                float nr;
                stk.pop(--sp, ref, nr);
                // its box passed with a larger-or-equal maxt; mint <= far does not depend on maxt
                if (STATS) st.boxes++;
                if (nr <= maxt) {
                    enter(ref);
                    break;
                }
            }
            if (k < 0 && cur < 0) {
                done = true;
                return;
            }
        }
#pragma unroll 1
        for (int it = 0; it < NH_NODES_PER_STEP && cur >= 0; ++it) {  // one wide node: test its child boxes
            float4 mnx, mny, mnz, mxx, mxy, mxz;
            int4 ref;
            if (cur < n_top) {  // the top of the tree, from the workgroup's LDS copy
                const float4 *n = top + kWideF4 * cur;
                mnx = n[0]; mny = n[1]; mnz = n[2]; mxx = n[3]; mxy = n[4]; mxz = n[5];
                ref = *reinterpret_cast<const int4 *>(&n[6]);
            } else {
                const float4 *n = tv.wnodes + (size_t)kWideF4 * cur;
                mnx = n[0]; mny = n[1]; mnz = n[2]; mxx = n[3]; mxy = n[4]; mxz = n[5];
                ref = *reinterpret_cast<const int4 *>(&n[6]);
            }
            float n0 = 0.f, n1 = 0.f, n2 = 0.f, n3 = 0.f;
            bool v0, v1, v2, v3;
            if (finite_r) {
#if NH_WIDE_PACKED_BOX
                box_test_finite_pair(f2{mnx.x, mnx.y}, f2{mny.x, mny.y}, f2{mnz.x, mnz.y}, f2{mxx.x, mxx.y},
                                     f2{mxy.x, mxy.y}, f2{mxz.x, mxz.y}, o.x, o.y, o.z, r.x, r.y, r.z, mint, maxt,
                                     v0, v1, n0, n1);
                box_test_finite_pair(f2{mnx.z, mnx.w}, f2{mny.z, mny.w}, f2{mnz.z, mnz.w}, f2{mxx.z, mxx.w},
                                     f2{mxy.z, mxy.w}, f2{mxz.z, mxz.w}, o.x, o.y, o.z, r.x, r.y, r.z, mint, maxt,
                                     v2, v3, n2, n3);
                v0 &= ref.x != kWideEmpty;
                v1 &= ref.y != kWideEmpty;
                v2 &= ref.z != kWideEmpty;
                v3 &= ref.w != kWideEmpty;
#else
                v0 = box_test_finite(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, o, r, mint, maxt, n0) & (ref.x != kWideEmpty);
                v1 = box_test_finite(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, o, r, mint, maxt, n1) & (ref.y != kWideEmpty);
                v2 = box_test_finite(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, o, r, mint, maxt, n2) & (ref.z != kWideEmpty);
                v3 = box_test_finite(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, o, r, mint, maxt, n3) & (ref.w != kWideEmpty);
#endif
            } else {
                v0 = ref.x != kWideEmpty && box_test(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, o, d, r, mint, maxt, n0);
                v1 = ref.y != kWideEmpty && box_test(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, o, d, r, mint, maxt, n1);
                v2 = ref.z != kWideEmpty && box_test(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, o, d, r, mint, maxt, n2);
                v3 = ref.w != kWideEmpty && box_test(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, o, d, r, mint, maxt, n3);
            }
            if (STATS) {
                st.nodes++;
                st.boxes += (ref.x != kWideEmpty) + (ref.y != kWideEmpty) + (ref.z != kWideEmpty) + (ref.w != kWideEmpty);
            }
            // Order of the hit children without moving them: rank_i = number of children before i
            // (wide_before: nearer first / slot order on ties, or slot order alone). cIJ (I < J) says
            // child I comes before child J; for two valid children exactly one of the two holds.
            const int c01 = wide_first<ORDERED>(v0, n0, v1, n1), c02 = wide_first<ORDERED>(v0, n0, v2, n2);
            const int c03 = wide_first<ORDERED>(v0, n0, v3, n3), c12 = wide_first<ORDERED>(v1, n1, v2, n2);
            const int c13 = wide_first<ORDERED>(v1, n1, v3, n3), c23 = wide_first<ORDERED>(v2, n2, v3, n3);
            const int rk0 = 3 - c01 - c02 - c03;
            const int rk1 = c01 + 2 - c12 - c13;
            const int rk2 = c02 + c12 + 1 - c23;
            const int rk3 = c03 + c13 + c23;
            const int nv = (int)v0 + (int)v1 + (int)v2 + (int)v3;
            if (nv == 0) {
                cur = -1;
            } else {
                // the nearest child is entered; child of rank r >= 1 is deferred at depth
                // sp + nv-1-r (farthest deepest, as pushing farthest first)
                stk.reserve(sp, nv - 1);
                const int top = sp + nv - 1;
                if (v0 && rk0) stk.put(top - rk0, ref.x, n0);
                if (v1 && rk1) stk.put(top - rk1, ref.y, n1);
                if (v2 && rk2) stk.put(top - rk2, ref.z, n2);
                if (v3 && rk3) stk.put(top - rk3, ref.w, n3);
                sp = top;
                enter((v0 && !rk0) ? ref.x : (v1 && !rk1) ? ref.y : (v2 && !rk2) ? ref.z : ref.w);
            }
        }
        if (k >= 0) {  // up to two primitives of the current leaf: records fetched together, tested as a pair
            const float4 a0 = tv.prims[3 * k], b0 = tv.prims[3 * k + 1], c0 = tv.prims[3 * k + 2];
            const float4 a1 = tv.prims[3 * k + 3], b1 = tv.prims[3 * k + 4], c1 = tv.prims[3 * k + 5];
#if NH_WIDE_PAIR
            f2 pt, pu, pv;
            bool ok0, ok1;
            tri_test_pair(a0, b0, c0, a1, b1, c1, o, d, mint, pt, pu, pv, ok0, ok1);
            if (prim(a0, c0, pt.x, pu.x, pv.x, ok0, st)) return;
            if (k >= 0) {
                if (prim(a1, c1, pt.y, pu.y, pv.y, ok1, st)) return;
            }
#else
            float t0, u0 = 0.f, v0 = 0.f;
            const bool ok0 = prim_is_tri(c0) && tri_test_nb(a0, b0, c0, o, d, mint, INFINITY, t0, u0, v0);
            if (prim(a0, c0, t0, u0, v0, ok0, st)) return;
            if (k >= 0) {
                float t1, u1 = 0.f, v1 = 0.f;
                const bool ok1 = prim_is_tri(c1) && tri_test_nb(a1, b1, c1, o, d, mint, INFINITY, t1, u1, v1);
                if (prim(a1, c1, t1, u1, v1, ok1, st)) return;
            }
#endif
        }
        if (k < 0 && cur < 0 && sp == 0) done = true;
    }

    // record k (a, c; for a triangle its pair-test results t, u, v, ok) against the current maxt, then
    // advance k; true when an any-hit query is answered
    NHD bool prim(const float4 &a, const float4 &c, float t, float u, float v, bool ok, TravStats &st) {
        if (STATS) st.prims++;
        bool hit;
        if (prim_is_tri(c)) {
            hit = ok & (t <= maxt);
        } else {
            u = v = 0.f;
            hit = sphere_test(a, o, d, mint, maxt, t);
        }
        if (hit) {
            if (is_any()) {
                found = true;
                done = true;
                return true;
            }
            if (t < maxt || k > best.k) {
                found = true;
                maxt = t;
                best.t = t;
                best.u = u;
                best.v = v;
                best.k = k;
            }
        }
        k = (__float_as_int(c.w) & kPrimLeafEnd) ? -1 : k + 1;
        return false;
    }

    NHD void enter(int ref) {
        if (ref >= 0) {
            cur = ref;
        } else {
            k = ~ref;
            cur = -1;
        }
    }
};

// ---------------------------------------------------------------------------------------------
// 8-wide traversal of the same tree (A/B against the 4-wide one, NH_WIDE8): nh_api.hip collapses the binary tree
// to 8 children per node by the same rule (the largest-area inner child replaced by its two children, slots in
// left-first DFS order, the descendants' own boxes -- no new boxes; the argument of Tracer4 carries over). A node
// is two 128-B lines, each laid out as a 4-wide node: children 0-3 in float4 [0..7], 4-7 in [8..15]. Both lines
// are loaded before either is tested, so one dependent fetch covers twice the children and a query takes about
// two thirds of the 4-wide dependent steps. Same answers as Tracer4 (smallest t, ties to the largest leaf-order
// position k); only the visit order of deferred children changes, which no answer depends on.
constexpr int kWide8F4 = 2 * kWideF4;

template <bool ORDERED, bool ANY, bool STATS, class Stack, bool RT = false>
struct Tracer8 {
    F3 o, d, r;
    float mint, maxt;
    int cur;  // wide node to visit next, or -1
    int k;    // primitive under test, or -1
    int sp;
    bool found, done;
    bool finite_r;
    bool any_q;  // RT: this lane's query is an any-hit query
    Hit best;

    NHD bool is_any() const { return RT ? any_q : ANY; }

    NHD void begin(const DScene &S, const Traversal &tv, F3 o_, F3 d_, float mint_, float maxt_, TravStats &st) {
        o = o_;
        d = d_;
        mint = mint_;
        maxt = maxt_;
        if (mint == kEps) mint = e_max(mint, mint * e_max(fabsf(o.x), e_max(fabsf(o.y), fabsf(o.z))));  // bvh.cpp:407-410
        best.k = -1;
        best.t = INFINITY;
        found = false;
        done = true;
        sp = 0;
        cur = -1;
        k = -1;
        if (S.root_kind == 0 || maxt < mint) return;
        r = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        finite_r = fabsf(r.x) < INFINITY && fabsf(r.y) < INFINITY && fabsf(r.z) < INFINITY;
        float near_t;
        if (STATS) st.boxes++;
        if (!box_test(S.root_min[0], S.root_min[1], S.root_min[2], S.root_max[0], S.root_max[1], S.root_max[2], o, d,
                      r, mint, maxt, near_t))
            return;
        done = false;
        if (S.root_kind == 2) k = tv.leaves[0].x;
        else cur = 0;
    }

    // the four children of one line: validity and entry distance
    NHD void line_tests(const float4 *n, bool *v, float *nn, int *ref) const {
        const float4 mnx = n[0], mny = n[1], mnz = n[2], mxx = n[3], mxy = n[4], mxz = n[5];
        const int4 rf = *reinterpret_cast<const int4 *>(&n[6]);
        ref[0] = rf.x; ref[1] = rf.y; ref[2] = rf.z; ref[3] = rf.w;
        nn[0] = nn[1] = nn[2] = nn[3] = 0.f;
        if (finite_r) {
            v[0] = box_test_finite(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, o, r, mint, maxt, nn[0]) & (rf.x != kWideEmpty);
            v[1] = box_test_finite(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, o, r, mint, maxt, nn[1]) & (rf.y != kWideEmpty);
            v[2] = box_test_finite(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, o, r, mint, maxt, nn[2]) & (rf.z != kWideEmpty);
            v[3] = box_test_finite(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, o, r, mint, maxt, nn[3]) & (rf.w != kWideEmpty);
        } else {
            v[0] = rf.x != kWideEmpty && box_test(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, o, d, r, mint, maxt, nn[0]);
            v[1] = rf.y != kWideEmpty && box_test(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, o, d, r, mint, maxt, nn[1]);
            v[2] = rf.z != kWideEmpty && box_test(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, o, d, r, mint, maxt, nn[2]);
            v[3] = rf.w != kWideEmpty && box_test(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, o, d, r, mint, maxt, nn[3]);
        }
    }

    NHD void step(const Traversal &tv, Stack &stk, TravStats &st) { step(tv, stk, st, nullptr, 0); }
    // top / n_top: an LDS copy of the first n_top 8-wide nodes (0: every node from tv.wnodes)
    NHD void step(const Traversal &tv, Stack &stk, TravStats &st, const float4 *top, int n_top) {
        if (k < 0 && cur < 0) {  // deferred children: the visit-time test against the current maxt
            while (sp > 0) {
                int ref;
                float nr;
                stk.pop(--sp, ref, nr);
                if (STATS) st.boxes++;
                if (nr <= maxt) {
                    enter(ref);
                    break;
                }
            }
            if (k < 0 && cur < 0) {
                done = true;
                return;
            }
        }
        if (cur >= 0) {  // one 8-wide node: both lines fetched, then the eight child boxes tested
            const float4 *n = cur < n_top ? top + kWide8F4 * cur : tv.wnodes + (size_t)kWide8F4 * cur;
            bool v[8];
            float nn[8];
            int ref[8];
            line_tests(n, v, nn, ref);
            line_tests(n + kWideF4, v + 4, nn + 4, ref + 4);
            if (STATS) {
                st.nodes++;
#pragma unroll
                for (int i = 0; i < 8; ++i) st.boxes += ref[i] != kWideEmpty;
            }
            // rank_i = number of valid children before child i (wide_first per pair: nearer first, slot order on ties)
            int rk[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) rk[i] = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = i + 1; j < 8; ++j) {
                    const int c = wide_first<ORDERED>(v[i], nn[i], v[j], nn[j]);
                    rk[j] += c;
                    rk[i] += 1 - c;
                }
            int nv = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) nv += (int)v[i];
            if (nv == 0) {
                cur = -1;
            } else {
                // the nearest child is entered; the child of rank r >= 1 is deferred at depth sp + nv-1-r
                stk.template reserve<7>(sp, nv - 1);
                const int top_i = sp + nv - 1;
                int first = ref[7];
#pragma unroll
                for (int i = 7; i >= 0; --i) {
                    if (v[i] && rk[i]) stk.put(top_i - rk[i], ref[i], nn[i]);
                    if (v[i] && !rk[i]) first = ref[i];
                }
                sp = top_i;
                enter(first);
            }
        }
        if (k >= 0) {  // up to two primitives of the current leaf: records fetched together, tested as a pair
            const float4 a0 = tv.prims[3 * k], b0 = tv.prims[3 * k + 1], c0 = tv.prims[3 * k + 2];
            const float4 a1 = tv.prims[3 * k + 3], b1 = tv.prims[3 * k + 4], c1 = tv.prims[3 * k + 5];
            f2 pt, pu, pv;
            bool ok0, ok1;
            tri_test_pair(a0, b0, c0, a1, b1, c1, o, d, mint, pt, pu, pv, ok0, ok1);
            if (prim(a0, c0, pt.x, pu.x, pv.x, ok0, st)) return;
            if (k >= 0) {
                if (prim(a1, c1, pt.y, pu.y, pv.y, ok1, st)) return;
            }
        }
        if (k < 0 && cur < 0 && sp == 0) done = true;
    }

    // record k against the current maxt, then advance k; true when an any-hit query is answered (as Tracer4::prim)
    NHD bool prim(const float4 &a, const float4 &c, float t, float u, float v, bool ok, TravStats &st) {
        if (STATS) st.prims++;
        bool hit;
        if (prim_is_tri(c)) {
            hit = ok & (t <= maxt);
        } else {
            u = v = 0.f;
            hit = sphere_test(a, o, d, mint, maxt, t);
        }
        if (hit) {
            if (is_any()) {
                found = true;
                done = true;
                return true;
            }
            if (t < maxt || k > best.k) {
                found = true;
                maxt = t;
                best.t = t;
                best.u = u;
                best.v = v;
                best.k = k;
            }
        }
        k = (__float_as_int(c.w) & kPrimLeafEnd) ? -1 : k + 1;
        return false;
    }

    NHD void enter(int ref) {
        if (ref >= 0) {
            cur = ref;
        } else {
            k = ~ref;
            cur = -1;
        }
    }
};

}  // namespace nhd
