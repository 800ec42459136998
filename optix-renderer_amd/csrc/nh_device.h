// Device-side math, sampling and shading for the gfx950 path_mis pipeline.
//
// Every routine restates a reference function (file:line in the comment) with the
// reference's fp32 rounding points: no contraction (file is compiled with
// -ffp-contract=off and the pragma below), 3-vector dot products grouped
// x0*y0 + (x1*y1 + x2*y2) as the reference's Eigen 3.3.8 emits them, Eigen's
// std::min/std::max ternaries (NaN behaviour included), and transcendentals
// evaluated in fp64 and rounded once (the reference calls the float libm, which is
// correctly rounded on the reference's inputs; a 1-ulp fp32 libm would diverge paths).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nhd {

constexpr float kEps = 1e-4f;
constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;

#define NHD __device__ __forceinline__

// lens-stream tables (DScene::lens_lo / lens_hi): rounds 256 h + l, h < kLensHi
constexpr int kLensLo = 256, kLensHi = 65536;

NHD float f_sin(float x) { return (float)sin((double)x); }
NHD float f_cos(float x) { return (float)cos((double)x); }

// sin and cos of one fp32 argument in [-8, 8] (every device call site passes a warp angle
// in [0, 2*pi]), evaluated in fp64 to ~1 ulp and rounded once: the fp32 results equal the
// correctly rounded sinf/cosf except on ~2^-29 of inputs. One shared reduction
// x = k*pi/2 + r (two-part Cody-Waite: k*PIO2_HI is exact for |k| < 2^20) and the classic
// degree-13 / degree-14 minimax kernels on |r| <= pi/4 (public-domain fdlibm constants).
// Much smaller than the general fp64 library routines (no large-argument path), which
// matters for the megakernel's register budget.
NHD void f_sincos(float xf, float &s_out, float &c_out) {
    const double x = (double)xf;
    const double k = __builtin_rint(x * 6.36619772367581382433e-01);  // 2/pi
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double z = r * r;
    const double sp = r + r * z * (-1.66666666666666324348e-01 +
                                   z * (8.33333333332248946124e-03 +
                                        z * (-1.98412698298579493134e-04 +
                                             z * (2.75573137070700676789e-06 +
                                                  z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)))));
    const double cp = 1.0 - 0.5 * z +
                      z * z * (4.16666666666666019037e-02 +
                               z * (-1.38888888888741095749e-03 +
                                    z * (2.48015872894767294178e-05 +
                                         z * (-2.75573143513906633035e-07 +
                                              z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const int q = ((int)k) & 3;
    double sv, cv;
    if (q == 0) { sv = sp; cv = cp; }
    else if (q == 1) { sv = cp; cv = -sp; }
    else if (q == 2) { sv = -sp; cv = -cp; }
    else { sv = -cp; cv = sp; }
    s_out = (float)sv;
    c_out = (float)cv;
}
#ifndef NH_AB_FAST_TRANSC  // cost attribution builds only (scripts/build_variant.sh): fp32 library forms, NOT exact
NHD float f_exp(float x) { return (float)exp((double)x); }
NHD float f_log(float x) { return (float)log((double)x); }
NHD float f_acos(float x) { return (float)acos((double)x); }
NHD float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
#else
NHD float f_exp(float x) { return expf(x); }
NHD float f_log(float x) { return logf(x); }
NHD float f_acos(float x) { return acosf(x); }
NHD float f_atan2(float y, float x) { return atan2f(y, x); }
#endif
NHD float f_sqrt(float x) { return __builtin_sqrtf(x); }  // correctly rounded (HIP default)
NHD float e_min(float a, float b) { return (b < a) ? b : a; }  // std::min
NHD float e_max(float a, float b) { return (a < b) ? b : a; }  // std::max

struct F3 {
    float x, y, z;
};
NHD F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
NHD F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
NHD F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
NHD F3 neg(F3 a) { return f3(-a.x, -a.y, -a.z); }
NHD F3 scl(float s, F3 a) { return f3(s * a.x, s * a.y, s * a.z); }
NHD F3 mulc(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
NHD F3 divs(F3 a, float s) { return f3(a.x / s, a.y / s, a.z / s); }
NHD float dot(F3 a, F3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
NHD F3 cross(F3 a, F3 b) { return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
NHD F3 normalized(F3 a) {
    float n = dot(a, a);
    if (n > 0.0f) {
        float s = f_sqrt(n);
        return f3(a.x / s, a.y / s, a.z / s);
    }
    return a;
}
NHD float max_coeff(F3 c) { return e_max(c.x, e_max(c.y, c.z)); }
NHD bool is_zero(F3 c) { return fabsf(c.x) <= kEps && fabsf(c.y) <= kEps && fabsf(c.z) <= kEps; }
NHD bool is_valid(F3 c) {
    return !(c.x < 0 || !isfinite(c.x) || c.y < 0 || !isfinite(c.y) || c.z < 0 || !isfinite(c.z));
}

// ---- pcg32 (ext/pcg32/pcg32.h:51-110) + the per-path seeding contract ------------
struct Rng {
    uint64_t state, inc;
    NHD uint32_t next_uint() {
        uint64_t old = state;
        state = old * kPcgMult + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31u));
    }
    NHD float next1d() { return __uint_as_float((next_uint() >> 9) | 0x3f800000u) - 1.0f; }
};
// pcg32() default state and stream (pcg32.h:29-30, :40) and pcg32::advance (pcg32.h:131-150): Brown's
// arbitrary-stride jump, O(log delta)
constexpr uint64_t kPcgDefaultState = 0x853c49e6748fea9bULL, kPcgDefaultStream = 0xda3e39cb94b95bdbULL;
NHD uint64_t pcg_advance(uint64_t state, uint64_t inc, uint64_t delta) {
    uint64_t cur_mult = kPcgMult, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
    while (delta > 0) {
        if (delta & 1) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta /= 2;
    }
    return acc_mult * state + acc_plus;
}
NHD uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// pcg32::seed(initstate = splitmix64(seed ^ pixel), initseq = sample)
NHD Rng path_rng(uint64_t seed, uint64_t pixel, uint64_t sample) {
    Rng r;
    r.state = 0u;
    r.inc = (sample << 1u) | 1u;
    r.next_uint();
    r.state += splitmix64(seed ^ pixel);
    r.next_uint();
    return r;
}
// path_rng with its splitmix64(seed ^ pixel) already formed (the splat reuses it over a pixel's rounds)
NHD Rng path_rng_h(uint64_t h, uint64_t sample) {
    Rng r;
    r.state = 0u;
    r.inc = (sample << 1u) | 1u;
    r.next_uint();
    r.state += h;
    r.next_uint();
    return r;
}
// The pixel jitter of a sample (render.cpp:441-442: the camera sample's first next2D): recomputed by the splat from
// the sample's seed instead of stored in its record
NHD void sample_jitter_h(uint64_t h, uint64_t sample, float &jx, float &jy) {
    Rng r = path_rng_h(h, sample);
    jx = r.next1d();
    jy = r.next1d();
}

// ---- scene records -----------------------------------------------------------
enum : int { SHAPE_MESH = 0, SHAPE_SPHERE = 1 };
enum : int { BSDF_DIFFUSE = 0, BSDF_MIRROR = 1, BSDF_DIELECTRIC = 2, BSDF_MICROFACET = 3 };
enum : int { EMITTER_AREA = 0, EMITTER_POINT = 1, EMITTER_ENVMAP = 2 };
enum : int { M_UNKNOWN = 0, M_SOLID_ANGLE = 1, M_DISCRETE = 2 };

struct alignas(16) DShape {
    int type, bsdf, emitter, v_off;
    int f_off, n_faces, has_n, has_uv;
    float cx, cy, cz, radius;
    int pdf_off;
    float pdf_norm;
    // bit 0: Intersection::uv is read (a textured diffuse albedo, or a normal map): hit_info computes uv only then;
    // bits 1+: 1 + the DScene::texs index of the shape's normal map (shape.cpp:138-147), 0 = none
    int tex_uv;
    int ef_off;  // emitting mesh without normals: its faces' first record in DScene::emit_faces, else -1
};
struct alignas(16) DBsdf {
    int type;
    float ar, ag, ab;      // diffuse albedo
    float alpha, int_ior, ext_ior, ks;
    float kr, kg, kb;      // microfacet kd
    int tex;               // diffuse: 1 + albedo texture index (DScene::texs), 0 = the constant albedo
};
// Texture<Color3f> albedo (nh_texture): consttexture.cpp / checkerboard.cpp / PNGTexture.cpp
enum : int { TEX_CONSTANT = 0, TEX_CHECKERBOARD = 1, TEX_PNG = 2 };
struct alignas(16) DTex {
    int type, w, h, spherical;
    float v1r, v1g, v1b, v2r;
    float v2g, v2b, dx, dy;
    float sx, sy, su, sv;
    float ou, ov;
    long long off;  // png: first texel in DScene::texels
    float rot[9];   // png spherical lookups: the eulerAngles rotation, row-major
    int linear;     // png with sRGB = false: normal-map texels, eval blends by intensity and normalizes
    float intensity;
    float pad;
};
struct alignas(16) DEmitter {
    int type, shape;
    float lr, lg, lb;
    float px, py, pz;
};

struct DScene {
    // BVH: 4 float4 per inner node, 3 float4 per primitive in leaf order
    const float4 *nodes;
    const float4 *prims;
    float root_min[3], root_max[3];
    int root_kind;  // 0 = empty scene, 1 = root inner node 0, 2 = root is a leaf
    int root_start, root_count;
    // geometry / materials
    const DShape *shapes;
    const DBsdf *bsdfs;
    const DEmitter *emitters;
    const float *emitter_cdf;
    int n_emitters;
    int integrator;  // 0 path_mis, 1 path_mats, 2-5 the direct integrators, 6 normals
    float ndir[3];   // normals: its `direction`
    const float *V, *N, *UV, *T, *BT;
    const uint32_t *F;
    const float *area_cdf;
    // emitting meshes without vertex normals, per face: (p0, n.x) (p1, n.y) (p2, n.z) with the face normal
    // normalized(cross(p1 - p0, p2 - p0)) of Mesh::sampleSurface (mesh.cpp:64-69), computed once at upload by the
    // same device arithmetic (nh_api.hip emit_face_kernel) instead of per light sample
    const float4 *emit_faces;
    // camera (perspective.cpp) and filter table (block.cpp)
    float s2c[16], c2w[16];
    // the pinhole ray origin (camera_ray with a (0, 0, 0) local origin: c2w * (0, 0, 0, 1), divided by its w), formed
    // once at upload by the same float operations in the same order
    float cam_o[3];
    float inv_w, inv_h, near_clip, far_clip;
    int width, height;
    // depth of field (perspective.cpp:114-130), on when lensRadius > Epsilon. The lens stream's state at a camera
    // ray's first draw (nh_shade.h lens_uniform): lens_pix[pixel] = advance by 2 x (the pixel's position within one
    // sample round of the serial render order: spiral blocks, x-major pixels) as (a, c); lens_lo[l] = advance by
    // 2 l W H; lens_hi[h] = the state at draw 2 * 256 h * W * H. lens_rtl: x = the second draw (g++'s order)
    int dof, lens_rtl;
    float lens_radius, focal_distance;
    const ulonglong2 *lens_pix, *lens_lo;
    const uint64_t *lens_hi;
    float filter_radius, lookup;
    int border;
    float table[33];
    // EnvMap (environmentmap.cpp) and its albedo texture (PNGTexture.cpp / ConstantTexture)
    int envmap;  // emitter index, or -1
    const float4 *env_rgba;
    const float *env_cdf;  // env_w * env_h + 1 entries
    const int *env_guide;  // 2^env_guide_bits + 1 entries: dpdf_sample_guided's brackets of env_cdf (nullptr: none)
    int env_guide_bits;
    int env_w, env_h, env_spherical, env_constant;
    float env_norm, env_su, env_sv, env_ou, env_ov;
    float env_r, env_g, env_b;
    float env_rot[9];  // spherical lookups: the png_texture's eulerAngles rotation, row-major
    // BSDF albedo textures (DBsdf::tex) and the png texels they index
    const DTex *texs;
    const float4 *texels;
    // 1: a light sample is always finite and never at a discrete-BSDF shading point (nh_api.hip, upload), so the
    // wavefront shade skips the light sample of a discrete BSDF sample (it provably adds +-0)
    int nee_finite;
    // isolated dielectric spheres the BVH upload marked (nh_traverse.h trace_next; 0: no ray tries the shortcut)
    int iso_spheres;
};

NHD F3 ldv(const float *a, uint32_t i) { return f3(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }

// ---- frames (frame.h, common.cpp:292-306) ---------------------------------------
struct Frame {
    F3 s, t, n;
};
NHD Frame frame_from_n(F3 a) {
    Frame f;
    f.n = a;
    F3 c;
    if (fabsf(a.x) > fabsf(a.y)) {
        float inv_len = 1.0f / f_sqrt(a.x * a.x + a.z * a.z);
        c = f3(a.z * inv_len, 0.0f, -a.x * inv_len);
    } else {
        float inv_len = 1.0f / f_sqrt(a.y * a.y + a.z * a.z);
        c = f3(0.0f, a.z * inv_len, -a.y * inv_len);
    }
    f.t = c;
    f.s = cross(c, a);
    return f;
}
NHD F3 to_local(const Frame &f, F3 v) { return f3(dot(v, f.s), dot(v, f.t), dot(v, f.n)); }
NHD F3 to_world(const Frame &f, F3 v) { return add(add(scl(v.x, f.s), scl(v.y, f.t)), scl(v.z, f.n)); }

// fresnel (common.cpp:308-338)
NHD float fresnel(float cos_i, float ext_ior, float int_ior) {
    float eta_i = ext_ior, eta_t = int_ior;
    if (ext_ior == int_ior) return 0.0f;
    if (cos_i < 0.0f) {
        float tmp = eta_i; eta_i = eta_t; eta_t = tmp;
        cos_i = -cos_i;
    }
    float eta = eta_i / eta_t, sin_t2 = eta * eta * (1 - cos_i * cos_i);
    if (sin_t2 > 1.0f) return 1.0f;
    float cos_t = f_sqrt(1.0f - sin_t2);
    float rs = (eta_i * cos_i - eta_t * cos_t) / (eta_i * cos_i + eta_t * cos_t);
    float rp = (eta_t * cos_i - eta_i * cos_t) / (eta_t * cos_i + eta_i * cos_t);
    return (rs * rs + rp * rp) / 2.0f;
}

// ---- warps (warp.cpp) -------------------------------------------------------------
NHD F3 cosine_hemisphere(float sx, float sy) {  // warp.cpp:48-52, 111-122
    float rho = f_sqrt(sx);
    float theta = sy * 2.0f * kPi;
    float st, ct;
    f_sincos(theta, st, ct);
    float x = rho * ct, y = rho * st;
    return f3(x, y, f_sqrt(1.f - (x * x + y * y)));
}
NHD F3 beckmann(float sx, float sy, float alpha) {  // warp.cpp:131-150
    float ls = f_log(1.f - sx);
    if (isinf(ls)) ls = 0;
    float tan2 = -alpha * alpha * ls;
    float phi = sy * 2.f * kPi;
    float ct = 1.f / f_sqrt(1 + tan2);
    float st = f_sqrt(1.f - ct * ct);
    float sphi, cphi;
    f_sincos(phi, sphi, cphi);
    F3 r = f3(st * cphi, st * sphi, ct);
    if (r.z < 0) r = neg(r);
    return r;
}
NHD F3 uniform_sphere(float sx, float sy) {  // warp.cpp:74-82
    F3 w;
    w.z = 2.0f * sx - 1.0f;
    float r = f_sqrt(1.0f - w.z * w.z);
    float sigma = 2.0f * kPi * sy;
    float ss, cs;
    f_sincos(sigma, ss, cs);
    w.x = r * cs;
    w.y = r * ss;
    return normalized(w);
}

// ---- BSDFs (src/bsdf) ---------------------------------------------------------------
NHD float tan_theta(F3 v) {
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return f_sqrt(temp) / v.z;
}
NHD float beckmann_d(const DBsdf &b, F3 m) {  // microfacet.cpp:60-66
    float temp = tan_theta(m) / b.alpha, ct = m.z, ct2 = ct * ct;
    return f_exp(-temp * temp) / (kPi * b.alpha * b.alpha * ct2 * ct2);
}
NHD float smith_g1(const DBsdf &b, F3 v, F3 m) {  // microfacet.cpp:69-89
    float tt = tan_theta(v);
    if (tt == 0.0f) return 1.0f;
    if (dot(m, v) * v.z <= 0) return 0.0f;
    float a = 1.0f / (b.alpha * tt);
    if (a >= 1.6f) return 1.0f;
    float a2 = a * a;
    return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
}
// alb: the diffuse albedo at the query's uv (m_albedo->eval(bRec.uv): the constant albedo, or its texture's
// value, nh_shade.h bsdf_albedo); unused by the other BSDFs
NHD F3 bsdf_eval(const DBsdf &b, F3 wi, F3 wo, int measure, F3 alb) {
    if (b.type == BSDF_DIFFUSE) {  // diffuse.cpp:94-103
        if (measure != M_SOLID_ANGLE || wi.z <= 0 || wo.z <= 0) return f3(0, 0, 0);
        return f3(alb.x * kInvPi, alb.y * kInvPi, alb.z * kInvPi);
    }
    if (b.type == BSDF_MICROFACET) {  // microfacet.cpp:92-105
        if (wo.z < 0.f) return f3(0, 0, 0);
        F3 wh = normalized(add(wi, wo));
        float den = b.ks * beckmann_d(b, wh) * fresnel(dot(wh, wi), b.ext_ior, b.int_ior) * smith_g1(b, wi, wh) *
                    smith_g1(b, wo, wh);
        float num = 4.f * wi.z * wo.z;
        float spec = den / num;
        return f3(b.kr * kInvPi + spec, b.kg * kInvPi + spec, b.kb * kInvPi + spec);
    }
    return f3(0, 0, 0);
}
NHD float bsdf_pdf(const DBsdf &b, F3 wi, F3 wo, int measure) {
    if (b.type == BSDF_DIFFUSE) {  // diffuse.cpp:106-120
        if (measure != M_SOLID_ANGLE || wi.z <= 0 || wo.z <= 0) return 0.0f;
        return kInvPi * wo.z;
    }
    if (b.type == BSDF_MICROFACET) {  // microfacet.cpp:108-119
        if (wo.z <= 0) return 0.f;
        F3 wh = normalized(add(wo, wi));
        float p1 = b.ks * beckmann_d(b, wh) * wh.z / (4.f * dot(wo, wh));
        float p2 = (1.f - b.ks) * wo.z * kInvPi;
        return p1 + p2;
    }
    return 0.0f;
}
// returns the sample weight; wo/measure out (wo stays (0,0,0) on early returns, vector.h:49)
NHD F3 bsdf_sample(const DBsdf &b, F3 wi, float sx, float sy, F3 &wo, int &measure, F3 alb) {
    wo = f3(0, 0, 0);
    measure = M_UNKNOWN;
    switch (b.type) {
        case BSDF_DIFFUSE:  // diffuse.cpp:123-140
            if (wi.z <= 0) return f3(0, 0, 0);
            measure = M_SOLID_ANGLE;
            wo = cosine_hemisphere(sx, sy);
            return alb;
        case BSDF_MIRROR:  // mirror.cpp:41-57
            if (wi.z <= 0) return f3(0, 0, 0);
            wo = f3(-wi.x, -wi.y, wi.z);
            measure = M_DISCRETE;
            return f3(1, 1, 1);
        case BSDF_DIELECTRIC: {  // dielectric.cpp:51-102
            float F = fresnel(wi.z, b.ext_ior, b.int_ior);
            measure = M_DISCRETE;
            if (sx < F) {
                wo = f3(-wi.x, -wi.y, wi.z);
                return f3(1, 1, 1);
            }
            F3 nrm = f3(0.f, 0.f, 1.f);
            float eta;
            if (wi.z < 0.f) {
                nrm = neg(nrm);
                eta = b.int_ior / b.ext_ior;
            } else {
                eta = b.ext_ior / b.int_ior;
            }
            float dn = dot(wi, nrm);
            F3 wt1 = scl(-eta, sub(wi, scl(dn, nrm)));
            double p2 = (double)dn * (double)dn;  // std::pow(float, 2) in double (exact)
            double root = sqrt(1.0 - (double)(eta * eta) * (1.0 - p2));
            F3 wt2 = scl((float)(-root), nrm);
            wo = add(wt1, wt2);
            float w = 1.f / eta / eta;
            return f3(w, w, w);
        }
        case BSDF_MICROFACET: {  // microfacet.cpp:122-148
            if (wi.z < 0) return f3(0, 0, 0);
            float s1 = sy;
            if (s1 < b.ks) {
                s1 /= b.ks;
                F3 wh = beckmann(sx, s1, b.alpha);
                wo = sub(scl(2.f, scl(dot(wi, wh), wh)), wi);
            } else {
                s1 = (s1 - b.ks) / (1.f - b.ks);
                wo = cosine_hemisphere(sx, s1);
            }
            if (wo.z <= 0.f) return f3(0, 0, 0);
            F3 e = bsdf_eval(b, wi, wo, M_UNKNOWN, alb);
            float p = bsdf_pdf(b, wi, wo, M_UNKNOWN);
            return f3(e.x / p * wo.z, e.y / p * wo.z, e.z / p * wo.z);
        }
    }
    return f3(0, 0, 0);
}

// DiscretePDF::sample (dpdf.h:124-130): lower_bound then clamp
// DiscretePDF::sample (dpdf.h): the first CDF entry not below x, minus one, clamped. [lo, hi): the search range of
// that first entry (the whole CDF, or a guide table's bracket, dpdf_sample_guided)
NHD int dpdf_search(const float *cdf, int n_entries, float x, int lo, int hi) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (cdf[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    int index = lo - 1;
    if (index < 0) index = 0;
    if (index > n_entries - 1) index = n_entries - 1;
    return index;
}
NHD int dpdf_sample(const float *cdf, int n_entries, float x) { return dpdf_search(cdf, n_entries, x, 0, n_entries + 1); }
// the emitter pick of the integrators (m_emitterPDF.sample): with one emitter DiscretePDF::sample's clamp returns 0 for
// every x, so the two dependent CDF reads of the search are skipped (the caller still draws x)
NHD int emitter_pick(const DScene &S, float x) {
    return S.n_emitters == 1 ? 0 : dpdf_sample(S.emitter_cdf, S.n_emitters, x);
}

// The same search bracketed by a guide table (Chen & Asau's cutpoint method), bit-identical: guide[j] is the first
// CDF index not below j / 2^bits (nh_api.hip env_guide), and the first index not below x is monotone in x, so for
// j = floor(x * 2^bits) -- exact, a power-of-two scaling of x in [0, 1) -- it lies in [guide[j], guide[j + 1]]:
// the binary search runs over that bracket (a few entries) instead of the whole CDF (21 dependent loads for
// C5's 1500 x 750 envmap).
NHD int dpdf_sample_guided(const float *cdf, int n_entries, float x, const int *guide, int bits) {
    const float s = x * (float)(1 << bits);
    int j = (int)s;
    if (!(s >= 0.f)) j = 0;  // (x in [0, 1) from next1d; NaN would take the full bracket below)
    if (j > (1 << bits) - 1) j = (1 << bits) - 1;
    const int lo = guide[j], hi = guide[j + 1];
    if (!(x >= 0.f && x < 1.f)) return dpdf_sample(cdf, n_entries, x);
    return dpdf_search(cdf, n_entries, x, lo, hi);
}

}  // namespace nhd
