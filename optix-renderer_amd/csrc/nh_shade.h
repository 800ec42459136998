// Shading-side device functions shared by the megakernel and the wavefront kernels:
// Mesh/Sphere::setHitInformation, area/point emitters, PerspectiveCamera::sampleRay.
#pragma once
#include "nh_traverse.h"

namespace nhd {

struct Its {  // Intersection (include/nori/shape.h:41-79); geoFrame only where needed
    F3 p;
    float u, v;
    Frame sh;
    int shape;
};

// the geometric frame of triangle record k, as staged (Traversal::frames)
__device__ __forceinline__ Frame staged_frame(const float4 *frames, int k) {
    const float4 fs = frames[3 * k], ft = frames[3 * k + 1], fn = frames[3 * k + 2];
    Frame f;
    f.s = f3(fs.x, fs.y, fs.z);
    f.t = f3(ft.x, ft.y, ft.z);
    f.n = f3(fn.x, fn.y, fn.z);
    return f;
}

__device__ __noinline__ F3 tex_eval(const DTex *texs, const float4 *texels, int ti, float u, float v);

// Mesh::setHitInformation (mesh.cpp:141-196) / Sphere::setHitInformation (sphere.cpp:96-124), with the shape's normal
// map (DShape::tex_uv >> 1) unless NMAP = false (the lean RR-ahead bounce kernel: scenes without textures)
#ifdef NH_AB_NO_NMAP  // cost attribution builds only (scripts/build_variant.sh): normal maps compiled out, NOT exact
#define NH_NMAP_ON false
#else
#define NH_NMAP_ON true
#endif
template <bool NMAP_ = true>
__device__ __forceinline__ void hit_info(const DScene &S, const Traversal &tv, const Hit &h, F3 o, F3 d, Its &its) {
    constexpr bool NMAP = NMAP_ && NH_NMAP_ON;
    const float4 a = tv.prims[3 * h.k], b = tv.prims[3 * h.k + 1];
    const int shape = __float_as_int(b.w);
    const DShape sh = S.shapes[shape];
    its.shape = shape;
    if (sh.type == SHAPE_SPHERE) {
        its.p = add(o, scl(h.t, d));
        F3 n = normalized(sub(its.p, f3(sh.cx, sh.cy, sh.cz)));
        // uv (two fp64-evaluated transcendentals) only matters to a textured albedo (bsdf_albedo) and a normal map,
        // its only readers: the specular chains that set the tail's length skip it
        its.u = its.v = 0.f;
        if (sh.tex_uv) {
            F3 mn = neg(n);
            float theta = f_acos(mn.z), phi = f_atan2(mn.y, mn.x);
            if (phi < 0) phi += 2 * kPi;
            its.u = phi / (2.f * kPi);
            its.v = theta / kPi;
        }
        F3 t = normalized(cross(f3(0, 0, 1), n));
        its.sh.s = t;
        its.sh.t = cross(n, t);
        its.sh.n = n;
        if (NMAP && (sh.tex_uv >> 1)) {  // sphere.cpp:115-121: the frame re-derived from the mapped normal
            const F3 nm = tex_eval(S.texs, S.texels, (sh.tex_uv >> 1) - 1, its.u, its.v);
            n = normalized(to_world(its.sh, nm));
            t = normalized(cross(f3(0, 0, 1), n));
            its.sh.s = t;
            its.sh.t = cross(n, t);
            its.sh.n = n;
        }
        return;
    }
    const float bx = 1 - (h.u + h.v), by = h.u, bz = h.v;
    const float4 c = tv.prims[3 * h.k + 2];
    const F3 p0 = f3(a.x, a.y, a.z), p1 = f3(b.x, b.y, b.z), p2 = f3(c.x, c.y, c.z);  // the mesh's vertices
    its.p = add(add(scl(bx, p0), scl(by, p1)), scl(bz, p2));
    its.u = h.u;
    its.v = h.v;
    if (!sh.has_uv && !sh.has_n) {
        its.sh = tv.frames ? staged_frame(tv.frames, h.k) : frame_from_n(normalized(cross(sub(p1, p0), sub(p2, p0))));
        return;
    }
    const int local = __float_as_int(a.w);
    const uint32_t *f = S.F + 3 * (size_t)(sh.f_off + local);
    const uint32_t i0 = sh.v_off + f[0], i1 = sh.v_off + f[1], i2 = sh.v_off + f[2];
    if (sh.has_uv && sh.tex_uv) {  // texture coordinates, read only by a textured albedo or a normal map
        its.u = bx * S.UV[2 * i0] + by * S.UV[2 * i1] + bz * S.UV[2 * i2];
        its.v = bx * S.UV[2 * i0 + 1] + by * S.UV[2 * i1 + 1] + bz * S.UV[2 * i2 + 1];
    }
    if (sh.has_n) {
        F3 nrm = normalized(add(add(scl(bx, ldv(S.N, i0)), scl(by, ldv(S.N, i1))), scl(bz, ldv(S.N, i2))));
        if (sh.has_uv) {
            its.sh.s = normalized(add(add(scl(bx, ldv(S.T, i0)), scl(by, ldv(S.T, i1))), scl(bz, ldv(S.T, i2))));
            its.sh.t = normalized(add(add(scl(bx, ldv(S.BT, i0)), scl(by, ldv(S.BT, i1))), scl(bz, ldv(S.BT, i2))));
            if (NMAP && (sh.tex_uv >> 1)) {  // mesh.cpp:173-183: normal = (TBN * m_normalMap->eval(uv)).normalized()
                const F3 nm = tex_eval(S.texs, S.texels, (sh.tex_uv >> 1) - 1, its.u, its.v);
                // TBN's columns are (tangent, bitangent, normal); Matrix3f * Vector3f per row x0*y0 + (x1*y1 + x2*y2)
                const F3 a = its.sh.s, b = its.sh.t;
                nrm = normalized(f3(a.x * nm.x + (b.x * nm.y + nrm.x * nm.z), a.y * nm.x + (b.y * nm.y + nrm.y * nm.z),
                                    a.z * nm.x + (b.z * nm.y + nrm.z * nm.z)));
            }
            its.sh.n = nrm;
        } else {
            its.sh = frame_from_n(nrm);
        }
    } else {
        its.sh = tv.frames ? staged_frame(tv.frames, h.k) : frame_from_n(normalized(cross(sub(p1, p0), sub(p2, p0))));
    }
}


// ---- EnvMap (environmentmap.cpp:73-169) + PNGTexture::eval (PNGTexture.cpp:125-160) ------------
// Nori's M_PI is a float constant (common.h:61), so all angle arithmetic is fp32.
__device__ __forceinline__ F3 spherical_direction(float theta, float phi) {  // common.cpp:270-281
    float st, ct, sp, cp;
    f_sincos(theta, st, ct);
    f_sincos(phi, sp, cp);
    return f3(st * cp, st * sp, ct);
}
__device__ __forceinline__ void spherical_coordinates(F3 v, float &theta, float &phi) {  // common.cpp:283-291
    theta = f_acos(v.z);
    phi = f_atan2(v.y, v.x);
    if (phi < 0) phi += 2 * kPi;
}
// Matrix3f * Vector3f as Eigen 3.3.8 evaluates it (row . v as x0*y0 + (x1*y1 + x2*y2)), m row-major
__device__ __forceinline__ F3 rot3(const float *m, F3 w) {
    return f3(m[0] * w.x + (m[1] * w.y + m[2] * w.z), m[3] * w.x + (m[4] * w.y + m[5] * w.z),
              m[6] * w.x + (m[7] * w.y + m[8] * w.z));
}

// static_cast<unsigned int>(float) / int(float) as the reference's x86-64 build executes them (cvttss2si: to 64
// bits and the low word for unsigned, |x| >= 2^63 or NaN -> 0; to 32 bits for int, out of range or NaN -> INT_MIN)
__device__ __forceinline__ unsigned x86_f2u(float x) { return fabsf(x) < 0x1p63f ? (unsigned)(long long)x : 0u; }
__device__ __forceinline__ int x86_f2i(float x) { return fabsf(x) < 0x1p31f ? (int)x : (int)0x80000000; }

// the texel lookup of PNGTexture::eval (PNGTexture.cpp:147-155): nearest texel, row 0 of the image first
__device__ __forceinline__ F3 png_lookup(const float4 *texels, unsigned W, unsigned H, float su, float sv, float u,
                                         float v) {
    const unsigned w = x86_f2u(u * su * (float)W);
    const unsigned h = H - x86_f2u(v * sv * (float)H);
    const float4 c = texels[(h * W + w) % (W * H)];
    return f3(c.x, c.y, c.z);
}

// the albedo texture of a diffuse BSDF at the hit's uv (diffuse.cpp:101/:139, m_albedo->eval(bRec.uv)):
// ConstantTexture, Checkerboard<Color3f> (checkerboard.cpp:29-47) or PNGTexture (PNGTexture.cpp:125-160)
__device__ __noinline__ F3 tex_eval(const DTex *texs, const float4 *texels, int ti, float u, float v) {
    const DTex t = texs[ti];
    if (t.type == TEX_CHECKERBOARD) {
        const float ox = u / t.sx - t.dx, oy = v / t.sy - t.dy;
        const int x = x86_f2i(ox) + (ox < 0.f), y = x86_f2i(oy) + (oy < 0.f);
        // (x + y) % 2 == 0 with the reference's wrap-around addition: the sum's low bit
        return (((unsigned)x + (unsigned)y) & 1u) == 0 ? f3(t.v1r, t.v1g, t.v1b) : f3(t.v2r, t.v2g, t.v2b);
    }
    if (t.type == TEX_PNG) {
        if (t.spherical) {
            const F3 wi = rot3(t.rot, spherical_direction(v * kPi, u * 2.f * kPi));
            float th, ph;
            spherical_coordinates(wi, th, ph);
            u = ph / (2.f * kPi);
            v = th / kPi;
        } else {
            u += t.ou;
            v += t.ov;
        }
        F3 c = png_lookup(texels + t.off, (unsigned)t.w, (unsigned)t.h, t.su, t.sv, u, v);
        if (t.linear) {  // sRGB = false, a normal map (PNGTexture.cpp:155-161): blend towards +z by intensity, normalize
            c.x = c.x * t.intensity;
            c.y = c.y * t.intensity;
            c.z = c.z * t.intensity + (1.f - t.intensity);
            c = normalized(c);
        }
        return c;
    }
    return f3(t.v1r, t.v1g, t.v1b);
}
// the diffuse albedo of BSDF b at uv: its constant colour unless it has a texture
__device__ __forceinline__ F3 bsdf_albedo(const DScene &S, const DBsdf &b, float u, float v) {
#ifndef NH_AB_NO_TEX  // cost attribution builds only (scripts/build_variant.sh): textures compiled out
    if (__builtin_expect(b.tex != 0, 0)) return tex_eval(S.texs, S.texels, b.tex - 1, u, v);
#endif
    return f3(b.ar, b.ag, b.ab);
}

__device__ __forceinline__ F3 env_tex(const DScene &S, float u, float v) {
    if (S.env_constant) {
        const float4 c = S.env_rgba[0];
        return f3(c.x, c.y, c.z);
    }
    if (S.env_spherical) {
        // rot * wi, Eigen's Matrix3f * Vector3f (eulerAngles = 0: the identity, signed zeros as Eigen produces them)
        const F3 wi = rot3(S.env_rot, spherical_direction(v * kPi, u * 2.f * kPi));
        float th, ph;
        spherical_coordinates(wi, th, ph);
        u = ph / (2.f * kPi);
        v = th / kPi;
    } else {
        u += S.env_ou;
        v += S.env_ov;
    }
    return png_lookup(S.env_rgba, (unsigned)S.env_w, (unsigned)S.env_h, S.env_su, S.env_sv, u, v);
}
__device__ __forceinline__ F3 env_eval(const DScene &S, F3 wi) {  // EnvMap::eval
    float th, ph;
    spherical_coordinates(wi, th, ph);
    const F3 c = env_tex(S, ph / (2.f * kPi), th / kPi);
    return f3(c.x * S.env_r, c.y * S.env_g, c.z * S.env_b);
}
__device__ __forceinline__ float env_pdf(const DScene &S, F3 wi) {  // EnvMap::pdf
    const float sphere_pdf = 0.25f / kPi;  // squareToUniformSpherePdf((1,0,0))
    if (S.env_w == 1 && S.env_h == 1) return sphere_pdf;
    const F3 c = env_eval(S, wi);
    const float lum = c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f;
    return lum * S.env_norm / sphere_pdf * (float)(unsigned)S.env_h * (float)(unsigned)S.env_w;
}

// AreaEmitter / PointLight / EnvMap (src/emitters/arealight.cpp:58-125, pointlight.cpp:47-78)
__device__ __forceinline__ float emitter_pdf(const DScene &S, const DEmitter &e, F3 ref, F3 p, F3 n, F3 wi) {
    if (e.type == EMITTER_ENVMAP) return env_pdf(S, wi);
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
    if (e.type == EMITTER_ENVMAP) {  // EnvMap::sample (environmentmap.cpp:73-101)
        const unsigned W = (unsigned)S.env_w, H = (unsigned)S.env_h;
        const unsigned elem = (unsigned)(S.env_guide ? dpdf_sample_guided(S.env_cdf, (int)(W * H), sx, S.env_guide,
                                                                          S.env_guide_bits)
                                                     : dpdf_sample(S.env_cdf, (int)(W * H), sx));
        const float i = (int)(elem / W) / (float)H, j = (int)(elem % W) / (float)W;
        const F3 v = (W == 1 && H == 1) ? uniform_sphere(sx, sy) : spherical_direction(j * kPi, i * 2.0f * kPi);
        es.p = f3(v.x * 1.f / kEps, v.y * 1.f / kEps, v.z * 1.f / kEps);
        es.n = neg(v);
        const F3 pr = sub(es.p, ref);
        es.wi = normalized(pr);
        es.so = es.p;
        es.sd = neg(es.wi);
        es.smint = kEps;
        es.smaxt = f_sqrt(dot(pr, pr)) - kEps;
        const float pdf = env_pdf(S, es.wi);
        if (pdf < kEps) return f3(0, 0, 0);
        const F3 ev = env_eval(S, es.wi);
        return f3(ev.x / pdf, ev.y / pdf, ev.z / pdf);
    }
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
        if (sh.ef_off >= 0) {  // the face's vertices and its normal, precomputed (DScene::emit_faces)
            const float4 *q = S.emit_faces + 3 * (size_t)(sh.ef_off + idt);
            const float4 q0 = q[0], q1 = q[1], q2 = q[2];
            p = add(add(scl(bu, f3(q0.x, q0.y, q0.z)), scl(bv, f3(q1.x, q1.y, q1.z))), scl(bw, f3(q2.x, q2.y, q2.z)));
            n = f3(q0.w, q1.w, q2.w);
        } else {
            const uint32_t *f = S.F + 3 * (size_t)(sh.f_off + idt);
            const uint32_t i0 = sh.v_off + f[0], i1 = sh.v_off + f[1], i2 = sh.v_off + f[2];
            const F3 p0 = ldv(S.V, i0), p1 = ldv(S.V, i1), p2 = ldv(S.V, i2);
            p = add(add(scl(bu, p0), scl(bv, p1)), scl(bw, p2));
            if (sh.has_n)
                n = normalized(add(add(scl(bu, ldv(S.N, i0)), scl(bv, ldv(S.N, i1))), scl(bw, ldv(S.N, i2))));
            else
                n = normalized(cross(sub(p1, p0), sub(p2, p0)));
        }
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

// The lens sample of a camera ray (perspective.cpp:118-122). The reference draws it from one static Independent
// sampler that is never prepare()d -- a default-state pcg32 (pcg32.h:40), two floats per sampleRay call, shared
// by every render thread. In the serial render order (sample rounds; blocks in BlockGenerator spiral order; a
// block's pixels x-major, render.cpp:281-347, :436, block.cpp:151-199, independent.cpp:85-99) camera ray
// k = round * W * H + lens_index[pixel] takes draws 2k and 2k + 1, which pcg32::advance reaches directly: every
// ray's lens sample is independent of how the rays are distributed over threads, blocks and ranks. (With several
// threads the reference's draws race, so only its single-thread order is reproducible: DESIGN.md §7.)
// The state at draw 2k is one affine map of the default state, composed from three table entries (nh_api.hip
// lens_tables: pcg32::advance is x -> a x + c mod 2^64, and advances compose and commute): two 64-bit multiply-adds
// instead of pcg_advance's O(log k) loop. Point2f(nextFloat(), nextFloat()) as g++ evaluates it (right to left,
// S.lens_rtl): x = draw 2k + 1, y = draw 2k.
NHD void lens_uniform(const DScene &S, int round, int pix, float &u, float &v) {
    const unsigned rr = (unsigned)round;  // < kLensLo * kLensHi (nh_render checks)
    const ulonglong2 lo = S.lens_lo[rr & (kLensLo - 1)], pa = S.lens_pix[pix];
    const uint64_t s_round = lo.x * S.lens_hi[rr / kLensLo] + lo.y;
    Rng r;
    r.inc = kPcgDefaultStream;
    r.state = pa.x * s_round + pa.y;
    const float a = r.next1d(), b = r.next1d();
    u = S.lens_rtl ? b : a;
    v = S.lens_rtl ? a : b;
}

// The thin-lens part of sampleRay (perspective.cpp:120-130): the local ray's origin on the lens and its direction
// through the focal point
__device__ __forceinline__ void camera_lens(const DScene &S, int round, int pix, F3 dl, F3 &lo, F3 &ld) {
    float su, sv;
    lens_uniform(S, round, pix, su, sv);
    // squareToUniformDisk (warp.cpp:48-52)
    const float rho = f_sqrt(su), theta = sv * 2.0f * kPi;
    float st, ct;
    f_sincos(theta, st, ct);
    const float lx = S.lens_radius * (rho * ct), ly = S.lens_radius * (rho * st);
    const float ft = S.focal_distance / dl.z;
    // pFocus = ray(ft) = o + ft * d with o = 0 (ray.h:80)
    const F3 pf = f3(0.0f + ft * dl.x, 0.0f + ft * dl.y, 0.0f + ft * dl.z);
    lo = f3(lx, ly, 0.f);
    ld = normalized(f3(pf.x - lo.x, pf.y - lo.y, pf.z - lo.z));
}

// PerspectiveCamera::sampleRay (perspective.cpp:97-141); `round` and `pix` place the ray in the serial order of the
// lens samples (used only with depth of field). DOF = false: the pinhole path alone, for the persistent traversal
// kernels, whose refill code the lens arithmetic pushed into spills (the host never runs them on a DOF scene)
template <bool DOF = true>
__device__ __forceinline__ void camera_ray(const DScene &S, float px, float py, F3 &o, F3 &d, float &mint,
                                           float &maxt, int round, int pix) {
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
    const F3 dl = normalized(f3(r[0] / r[3], r[1] / r[3], r[2] / r[3]));
    F3 lo = f3(0.0f, 0.0f, 0.0f), ld = dl;  // local ray
    if (DOF && S.dof) {
        camera_lens(S, round, pix, dl, lo, ld);
        float ow[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float acc = S.c2w[4 * i] * lo.x;
            acc = acc + S.c2w[4 * i + 1] * lo.y;
            acc = acc + S.c2w[4 * i + 2] * lo.z;
            acc = acc + S.c2w[4 * i + 3] * 1.0f;
            ow[i] = acc;
        }
        o = f3(ow[0] / ow[3], ow[1] / ow[3], ow[2] / ow[3]);
    } else {
        o = f3(S.cam_o[0], S.cam_o[1], S.cam_o[2]);  // the same expression for lo = (0, 0, 0), formed at upload
    }
    const float *w = S.c2w;
    d = f3(w[0] * ld.x + (w[1] * ld.y + w[2] * ld.z), w[4] * ld.x + (w[5] * ld.y + w[6] * ld.z),
           w[8] * ld.x + (w[9] * ld.y + w[10] * ld.z));
    // the clip range follows the pinhole direction (perspective.cpp:135-137)
    const float inv_z = 1.0f / dl.z;
    mint = S.near_clip * inv_z;
    maxt = S.far_clip * inv_z;
}

}  // namespace nhd
