// TEST INFRASTRUCTURE ONLY -- see nori_oracle.h for the pinning statement.
//
// CPU restatement of Nori's path_mis hot path, following the reference source
// structure function by function (file:line cited at each piece). Build flags:
// g++ -O2 -ffp-contract=off (no FMA contraction, no fast-math), so every fp32
// operation rounds exactly where the reference's scalar code does.
//
// Evaluation-order conventions (how the reference's vendored Eigen 3.3.8 evaluates,
// measured in this container with a probe against ext/eigen):
//   - 3-vector dot / squaredNorm / 3x3 mat-vec:  x0*y0 + (x1*y1 + x2*y2)
//   - cwise chains evaluate left to right exactly as written in the source
//   - normalized() divides each component by sqrt(squaredNorm) (if > 0)
//   - maxCoeff over 3: f(c0, f(c1, c2)) with f(a,b) = a < b ? b : a
// Transcendentals: the reference's translation units see the float overloads
// (IlmBase's ImathPlatform.h includes <math.h>), i.e. sinf/cosf/expf/logf/...;
// these are evaluated here as fp64 and rounded once (measured equal to glibc's float
// libm by the survey). std::pow(float, int) promotes to double
// in C++11 and is kept in double where the reference keeps it (dielectric.cpp:90,
// sphere.cpp:130-137).
#include "nori_oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <memory>
#include <thread>
#include <vector>

namespace {

constexpr float kEps = 1e-4f;                          // common.h:56 Epsilon
constexpr float kPi = 3.14159265358979323846f;         // common.h:61 M_PI (float)
constexpr float kInvPi = 0.31830988618379067154f;      // common.h:62
constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;   // pcg32.h:31
constexpr uint64_t kPcgState = 0x853c49e6748fea9bULL;  // pcg32.h:29
constexpr uint64_t kPcgStream = 0xda3e39cb94b95bdbULL; // pcg32.h:30

// fp64-evaluated, singly rounded float transcendentals
inline float f_sin(float x) { return (float)std::sin((double)x); }
inline float f_cos(float x) { return (float)std::cos((double)x); }
inline float f_exp(float x) { return (float)std::exp((double)x); }
inline float f_log(float x) { return (float)std::log((double)x); }
inline float f_acos(float x) { return (float)std::acos((double)x); }
inline float f_atan2(float y, float x) { return (float)std::atan2((double)y, (double)x); }
inline float f_sqrt(float x) { return std::sqrt(x); }  // IEEE correctly rounded

// ---------------------------------------------------------------------------
// pcg32 (ext/pcg32/pcg32.h:38-110)
// ---------------------------------------------------------------------------
struct Pcg32 {
    uint64_t state = kPcgState, inc = kPcgStream;
    void seed(uint64_t initstate, uint64_t initseq) {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        next_uint();
        state += initstate;
        next_uint();
    }
    uint32_t next_uint() {
        uint64_t old = state;
        state = old * kPcgMult + inc;
        uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    float next_float() {
        uint32_t u = (next_uint() >> 9) | 0x3f800000u;
        float f;
        std::memcpy(&f, &u, 4);
        return f - 1.0f;
    }
    void advance(int64_t delta_) {  // pcg32.h:131-150
        uint64_t cur_mult = kPcgMult, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
        uint64_t delta = (uint64_t)delta_;
        while (delta > 0) {
            if (delta & 1) {
                acc_mult *= cur_mult;
                acc_plus = acc_plus * cur_mult + cur_plus;
            }
            cur_plus = (cur_mult + 1) * cur_plus;
            cur_mult *= cur_mult;
            delta /= 2;
        }
        state = acc_mult * state + acc_plus;
    }
};

inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Per-(pixel, sample) seeding contract shared with the GPU path:
//   pcg32.seed(initstate = splitmix64(seed ^ pixel_index), initseq = sample_index)
inline void path_seed(Pcg32 &r, uint64_t seed, uint64_t pixel, uint64_t sample) {
    r.seed(splitmix64(seed ^ pixel), sample);
}

struct Sampler {  // Independent (src/samplers/independent.cpp:69-79)
    Pcg32 rng;
    float next1d() { return rng.next_float(); }
    void next2d(float &a, float &b) {
        a = rng.next_float();
        b = rng.next_float();
    }
};

// ---------------------------------------------------------------------------
// vector math in Eigen's evaluation order
// ---------------------------------------------------------------------------
struct V3 {
    float x, y, z;
};
inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
inline V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
inline V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline V3 cmul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
inline float dot(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
inline float sqnorm(V3 a) { return dot(a, a); }
inline float norm(V3 a) { return f_sqrt(sqnorm(a)); }
inline V3 normalized(V3 a) {
    float n = sqnorm(a);
    if (n > 0.0f) return a / f_sqrt(n);
    return a;
}
inline V3 cross(V3 a, V3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline float eig_max(float a, float b) { return a < b ? b : a; }  // std::max / numext::maxi
inline float max_coeff(V3 c) { return eig_max(c.x, eig_max(c.y, c.z)); }
inline bool is_zero(V3 c) {  // Eigen isZero(Epsilon): all |c_i| <= prec
    return std::fabs(c.x) <= kEps && std::fabs(c.y) <= kEps && std::fabs(c.z) <= kEps;
}
inline bool is_valid(V3 c) {  // Color3f::isValid (common.cpp:254-263)
    for (float v : {c.x, c.y, c.z})
        if (v < 0 || !std::isfinite(v)) return false;
    return true;
}
inline float luminance(V3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }

struct Ray {  // Ray3f (include/nori/ray.h)
    V3 o, d, drcp;
    float mint, maxt;
};
inline Ray make_ray(V3 o, V3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.mint = kEps;
    r.maxt = std::numeric_limits<float>::infinity();
    r.drcp = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    return r;
}
inline Ray make_ray(V3 o, V3 d, float mint, float maxt) {
    Ray r = make_ray(o, d);
    r.mint = mint;
    r.maxt = maxt;
    return r;
}

// coordinateSystem (common.cpp:292-306) / Frame (frame.h)
void coordinate_system(V3 a, V3 &b, V3 &c) {
    if (std::fabs(a.x) > std::fabs(a.y)) {
        float inv_len = 1.0f / f_sqrt(a.x * a.x + a.z * a.z);
        c = mk(a.z * inv_len, 0.0f, -a.x * inv_len);
    } else {
        float inv_len = 1.0f / f_sqrt(a.y * a.y + a.z * a.z);
        c = mk(0.0f, a.z * inv_len, -a.y * inv_len);
    }
    b = cross(c, a);
}
struct Frame {
    V3 s, t, n;
    static Frame from_n(V3 n) {
        Frame f;
        f.n = n;
        coordinate_system(n, f.s, f.t);
        return f;
    }
    V3 to_local(V3 v) const { return mk(dot(v, s), dot(v, t), dot(v, n)); }
    V3 to_world(V3 v) const { return s * v.x + t * v.y + n * v.z; }
};

// fresnel (common.cpp:308-338)
float fresnel(float cos_i, float ext_ior, float int_ior) {
    float eta_i = ext_ior, eta_t = int_ior;
    if (ext_ior == int_ior) return 0.0f;
    if (cos_i < 0.0f) {
        std::swap(eta_i, eta_t);
        cos_i = -cos_i;
    }
    float eta = eta_i / eta_t, sin_t2 = eta * eta * (1 - cos_i * cos_i);
    if (sin_t2 > 1.0f) return 1.0f;
    float cos_t = f_sqrt(1.0f - sin_t2);
    float rs = (eta_i * cos_i - eta_t * cos_t) / (eta_i * cos_i + eta_t * cos_t);
    float rp = (eta_t * cos_i - eta_i * cos_t) / (eta_t * cos_i + eta_i * cos_t);
    return (rs * rs + rp * rp) / 2.0f;
}

// ---------------------------------------------------------------------------
// warps (src/utils/warp.cpp)
// ---------------------------------------------------------------------------
// NO_UNQUALIFIED_DOUBLE=1: unqualified sqrt/cos/sin/log on float arguments in warp.cpp /
// sphere.cpp resolve to the C double functions (a build whose ImathPlatform.h does not pull
// the C++ <math.h> overloads into the global namespace); default 0: float overloads (IlmBase's
// ImathPlatform.h includes <math.h>). Only the rounding points differ.
#ifndef NO_UNQUALIFIED_DOUBLE
#define NO_UNQUALIFIED_DOUBLE 0
#endif
void square_to_uniform_disk(float sx, float sy, float &x, float &y) {  // warp.cpp:48-52
    float rho = f_sqrt(sx);
    float theta = sy * 2.0f * kPi;
#if NO_UNQUALIFIED_DOUBLE
    x = (float)((double)rho * std::cos((double)theta));
    y = (float)((double)rho * std::sin((double)theta));
#else
    x = rho * f_cos(theta);
    y = rho * f_sin(theta);
#endif
}
V3 square_to_cosine_hemisphere(float sx, float sy) {  // warp.cpp:111-122
    float x, y;
    square_to_uniform_disk(sx, sy, x, y);
    return mk(x, y, f_sqrt(1.f - (x * x + y * y)));
}
V3 square_to_beckmann(float sx, float sy, float alpha) {  // warp.cpp:131-150
    float log_sample = f_log(1.f - sx);
    if (std::isinf(log_sample)) log_sample = 0;
    float tan2 = -alpha * alpha * log_sample;
    float phi = sy * 2.f * kPi;
#if NO_UNQUALIFIED_DOUBLE
    float cos_t = (float)(1.f / std::sqrt((double)(1 + tan2)));
#else
    float cos_t = 1.f / f_sqrt(1 + tan2);
#endif
    float sin_t = f_sqrt(1.f - cos_t * cos_t);
    V3 res = mk(sin_t * f_cos(phi), sin_t * f_sin(phi), cos_t);
    if (res.z < 0) res = -res;
    return res;
}
V3 square_to_uniform_triangle(float sx, float sy) {  // warp.cpp:162-166
    float su1 = std::sqrt(sx);
    float u = 1.f - su1, v = sy * su1;
    return mk(u, v, 1.f - u - v);
}
V3 square_to_uniform_sphere(float sx, float sy) {  // warp.cpp:74-82
    V3 w;
    w.z = 2.0f * sx - 1.0f;
    float r = f_sqrt(1.0f - w.z * w.z);
    float sigma = 2.0f * kPi * sy;
#if NO_UNQUALIFIED_DOUBLE
    w.x = (float)((double)r * std::cos((double)sigma));
    w.y = (float)((double)r * std::sin((double)sigma));
#else
    w.x = r * f_cos(sigma);
    w.y = r * f_sin(sigma);
#endif
    return normalized(w);
}

// ---------------------------------------------------------------------------
// BSDFs (src/bsdf/*.cpp), local frame
// ---------------------------------------------------------------------------
enum Measure { EUnknown = 0, ESolidAngle = 1, EDiscrete = 2 };
struct BRec {
    V3 wi, wo = mk(0, 0, 0);  // Nori vectors zero-initialise (vector.h:49)
    float eta = 1.0f;
    Measure measure = EUnknown;
    // BSDFQueryRecord::uv (bsdf.h:58), set to its.uv by every integrator (path_mis.cpp:92/:110, path_mats.cpp:64,
    // direct*.cpp), and the scene whose texture table a textured albedo indexes
    float u = 0.f, v = 0.f;
    const ::no_scene *scene = nullptr;
};

// m_albedo->eval(bRec.uv) (diffuse.cpp:101, :139): the constant albedo or the BSDF's texture
V3 diffuse_albedo(const nh_bsdf &b, const BRec &r);

inline float tan_theta(V3 v) {  // frame.h:76-82
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return f_sqrt(temp) / v.z;
}
float eval_beckmann(const nh_bsdf &b, V3 m) {  // microfacet.cpp:60-66
    float temp = tan_theta(m) / b.alpha, ct = m.z, ct2 = ct * ct;
    return f_exp(-temp * temp) / (kPi * b.alpha * b.alpha * ct2 * ct2);
}
float smith_g1(const nh_bsdf &b, V3 v, V3 m) {  // microfacet.cpp:69-89
    float tt = tan_theta(v);
    if (tt == 0.0f) return 1.0f;
    if (dot(m, v) * v.z <= 0) return 0.0f;
    float a = 1.0f / (b.alpha * tt);
    if (a >= 1.6f) return 1.0f;
    float a2 = a * a;
    return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
}

V3 bsdf_eval(const nh_bsdf &b, const BRec &r) {
    switch (b.type) {
        case NH_BSDF_DIFFUSE:  // diffuse.cpp:94-103
            if (r.measure != ESolidAngle || r.wi.z <= 0 || r.wo.z <= 0) return mk(0, 0, 0);
            return diffuse_albedo(b, r) * kInvPi;
        case NH_BSDF_MICROFACET: {  // microfacet.cpp:92-105
            if (r.wo.z < 0.f) return mk(0, 0, 0);
            V3 wh = normalized(r.wi + r.wo);
            float den = b.ks * eval_beckmann(b, wh) * fresnel(dot(wh, r.wi), b.ext_ior, b.int_ior) *
                        smith_g1(b, r.wi, wh) * smith_g1(b, r.wo, wh);
            float num = 4.f * r.wi.z * r.wo.z;
            float spec = den / num;
            return mk(b.kd[0] * kInvPi + spec, b.kd[1] * kInvPi + spec, b.kd[2] * kInvPi + spec);
        }
        default:  // mirror / dielectric: discrete, eval == 0
            return mk(0, 0, 0);
    }
}
float bsdf_pdf(const nh_bsdf &b, const BRec &r) {
    switch (b.type) {
        case NH_BSDF_DIFFUSE:  // diffuse.cpp:106-120
            if (r.measure != ESolidAngle || r.wi.z <= 0 || r.wo.z <= 0) return 0.0f;
            return kInvPi * r.wo.z;
        case NH_BSDF_MICROFACET: {  // microfacet.cpp:108-119
            if (r.wo.z <= 0) return 0.f;
            V3 wh = normalized(r.wo + r.wi);
            float part1 = b.ks * eval_beckmann(b, wh) * wh.z / (4.f * dot(r.wo, wh));
            float part2 = (1.f - b.ks) * r.wo.z * kInvPi;
            return part1 + part2;
        }
        default:
            return 0.0f;
    }
}
V3 bsdf_sample(const nh_bsdf &b, BRec &r, float sx, float sy) {
    switch (b.type) {
        case NH_BSDF_DIFFUSE:  // diffuse.cpp:123-140
            if (r.wi.z <= 0) return mk(0, 0, 0);
            r.measure = ESolidAngle;
            r.wo = square_to_cosine_hemisphere(sx, sy);
            r.eta = 1.0f;
            return diffuse_albedo(b, r);
        case NH_BSDF_MIRROR:  // mirror.cpp:41-57
            if (r.wi.z <= 0) return mk(0, 0, 0);
            r.wo = mk(-r.wi.x, -r.wi.y, r.wi.z);
            r.measure = EDiscrete;
            r.eta = 1.0f;
            return mk(1, 1, 1);
        case NH_BSDF_DIELECTRIC: {  // dielectric.cpp:51-102
            float cos_wi = r.wi.z;
            float F = fresnel(cos_wi, b.ext_ior, b.int_ior);
            r.measure = EDiscrete;
            if (sx < F) {
                r.wo = -r.wi;
                r.wo.z = r.wi.z;
                r.eta = 1.0f;
                return mk(1, 1, 1);
            }
            V3 normal = mk(0.f, 0.f, 1.f);
            if (cos_wi < 0.f) {
                normal = -normal;
                r.eta = b.int_ior / b.ext_ior;
            } else {
                r.eta = b.ext_ior / b.int_ior;
            }
            float dn = dot(r.wi, normal);
            V3 wt1 = -r.eta * (r.wi - dn * normal);
            double p2 = std::pow((double)dn, 2);
            double root = std::sqrt(1.0 - (double)(r.eta * r.eta) * (1.0 - p2));
            V3 wt2 = (float)(-root) * normal;
            r.wo = wt1 + wt2;
            return mk(1.f / r.eta / r.eta, 1.f / r.eta / r.eta, 1.f / r.eta / r.eta);
        }
        case NH_BSDF_MICROFACET: {  // microfacet.cpp:122-148
            if (r.wi.z < 0) return mk(0, 0, 0);
            float s0 = sx, s1 = sy;
            if (s1 < b.ks) {
                s1 /= b.ks;
                V3 wh = square_to_beckmann(s0, s1, b.alpha);
                r.wo = 2.f * (dot(r.wi, wh) * wh) - r.wi;
            } else {
                s1 = (s1 - b.ks) / (1.f - b.ks);
                r.wo = square_to_cosine_hemisphere(s0, s1);
            }
            if (r.wo.z <= 0.f) return mk(0, 0, 0);
            V3 e = bsdf_eval(b, r);
            float p = bsdf_pdf(b, r);
            return (e / p) * r.wo.z;
        }
    }
    return mk(0, 0, 0);
}

// ---------------------------------------------------------------------------
// scene
// ---------------------------------------------------------------------------
struct Its {  // Intersection (shape.h:41-79)
    V3 p;
    float t;
    float u, v;
    Frame sh, geo;
    int shape = -1;
};

struct BNode {  // BVHNode (bvh.h:127-165)
    uint32_t w0, w1;
    float mn[3], mx[3];
    bool leaf() const { return (w0 & 1u) != 0; }
    uint32_t size() const { return w0 >> 1; }
};

}  // namespace

struct no_scene {
    nh_camera cam;
    nh_filter filter;
    int integrator;
    float normals_dir[3];
    std::vector<nh_shape> shapes;
    std::vector<nh_bsdf> bsdfs;
    std::vector<nh_emitter> emitters;
    std::vector<float> emitter_cdf;
    std::vector<V3> V, N, T, BT;
    std::vector<float> UV;
    std::vector<uint32_t> F;
    std::vector<float> area_cdf;
    int envmap = -1;              // emitter index of the EnvMap, or -1
    nh_envmap env{};              // scalar parameters (pointers below)
    std::vector<float> env_rgba;  // PNGTexture::data
    std::vector<float> env_cdf;   // EnvMap::calculateProbs, recomputed here (no_env_cdf)
    std::vector<nh_texture> textures;  // BSDF albedo textures (nh_bsdf.albedo_texture = index + 1)
    std::vector<float> texels;         // RGBA texels of the png textures
    std::vector<uint32_t> shape_offset;
    std::vector<BNode> nodes;
    std::vector<uint32_t> indices;
    float bmin[3], bmax[3];
};

namespace {

// ---- primitive queries (src/shapes/mesh.cpp, sphere.cpp) ------------------
inline uint32_t find_shape(const no_scene &s, uint32_t &idx) {  // bvh.h:105-109
    auto it = std::lower_bound(s.shape_offset.begin(), s.shape_offset.end(), idx + 1) - 1;
    idx -= *it;
    return (uint32_t)(it - s.shape_offset.begin());
}
inline void tri_verts(const no_scene &s, const nh_shape &sh, uint32_t i, V3 &p0, V3 &p1, V3 &p2, uint32_t *vi = nullptr) {
    const uint32_t *f = &s.F[3 * ((size_t)sh.f_offset + i)];
    p0 = s.V[sh.v_offset + f[0]];
    p1 = s.V[sh.v_offset + f[1]];
    p2 = s.V[sh.v_offset + f[2]];
    if (vi) { vi[0] = sh.v_offset + f[0]; vi[1] = sh.v_offset + f[1]; vi[2] = sh.v_offset + f[2]; }
}

bool mesh_intersect(const no_scene &s, const nh_shape &sh, uint32_t i, const Ray &ray, float &u, float &v, float &t) {
    V3 p0, p1, p2;  // mesh.cpp:101-139
    tri_verts(s, sh, i, p0, p1, p2);
    V3 e1 = p1 - p0, e2 = p2 - p0;
    V3 pvec = cross(ray.d, e2);
    float det = dot(e1, pvec);
    if (det > -1e-8f && det < 1e-8f) return false;
    float inv_det = 1.0f / det;
    V3 tvec = ray.o - p0;
    u = dot(tvec, pvec) * inv_det;
    if (u < 0.0 || u > 1.0) return false;
    V3 qvec = cross(tvec, e1);
    v = dot(ray.d, qvec) * inv_det;
    if (v < 0.0 || u + v > 1.0) return false;
    t = dot(e2, qvec) * inv_det;
    return t >= ray.mint && t <= ray.maxt;
}

bool sphere_intersect(const nh_shape &sh, const Ray &ray, float &t) {  // sphere.cpp:67-94
    V3 c = mk(sh.center[0], sh.center[1], sh.center[2]);
    V3 L = ray.o - c;
    float a = dot(ray.d, ray.d);
    float b = 2.f * dot(ray.d, L);
    float cc = dot(L, L) - sh.radius * sh.radius;
    float discr = b * b - 4.f * a * cc;
    if (discr < 0.f) return false;
#if NO_UNQUALIFIED_DOUBLE
    const float tmin = (float)(((double)(-b) - std::sqrt((double)discr)) / 2 / (double)a);
    const float tmax = (float)(((double)(-b) + std::sqrt((double)discr)) / 2 / (double)a);
#else
    const float tmin = (-b - f_sqrt(discr)) / 2 / a;
    const float tmax = (-b + f_sqrt(discr)) / 2 / a;
#endif
    if (ray.mint <= tmin && ray.maxt >= tmin) { t = tmin; return true; }
    if (ray.mint <= tmax && ray.maxt >= tmax) { t = tmax; return true; }
    return false;
}

V3 texture_eval(const no_scene &s, const nh_texture &t, float u, float v);

// mesh.cpp:176-182: Eigen::Matrix3f TBN; TBN << aTangent, aBitangent, normal (columns);
// normal = (TBN * m_normalMap->eval(its.uv)).normalized(), each row of the product x0*y0 + (x1*y1 + x2*y2)
V3 tbn_normal(V3 tg, V3 bt, V3 nrm, V3 nm) {
    return normalized(mk(tg.x * nm.x + (bt.x * nm.y + nrm.x * nm.z), tg.y * nm.x + (bt.y * nm.y + nrm.y * nm.z),
                         tg.z * nm.x + (bt.z * nm.y + nrm.z * nm.z)));
}
// sphere.cpp:117-120: n = its.shFrame.toWorld(eval(uv)).normalized() (Frame::toWorld = s * x + t * y + n * z,
// frame.h:61-63); t = (Vector3f(0,0,1).cross(n)).normalized(); b = n.cross(t)
Frame sphere_reframe(const Frame &f, V3 nm) {
    Frame r;
    r.n = normalized(f.s * nm.x + f.t * nm.y + f.n * nm.z);
    r.s = normalized(cross(mk(0, 0, 1), r.n));
    r.t = cross(r.n, r.s);
    return r;
}
// PNGTexture::eval's !sRgb branch (PNGTexture.cpp:155-161): out.matrix().normalize() after the intensity blend
V3 normal_blend(V3 out, float intensity) {
    out.x = out.x * intensity;
    out.y = out.y * intensity;
    out.z = out.z * intensity + (1.f - intensity);
    return normalized(out);
}

void set_hit_information(const no_scene &s, uint32_t shape, uint32_t prim, const Ray &ray, Its &its) {
    const nh_shape &sh = s.shapes[shape];
    its.shape = (int)shape;
    if (sh.type == NH_SHAPE_SPHERE) {  // sphere.cpp:96-124
        V3 c = mk(sh.center[0], sh.center[1], sh.center[2]);
        its.p = ray.o + its.t * ray.d;
        V3 n = normalized(its.p - c);
        V3 mn = -n;
        float theta = f_acos(mn.z), phi = f_atan2(mn.y, mn.x);
        if (phi < 0) phi += 2 * kPi;
        its.u = phi / (2.f * kPi);
        its.v = theta / kPi;
        its.geo = Frame::from_n(n);
        V3 t = normalized(cross(mk(0, 0, 1), n));
        V3 b = cross(n, t);
        its.sh.s = t;
        its.sh.t = b;
        its.sh.n = n;
        if (sh.normal_map)  // sphere.cpp:115-121
            its.sh = sphere_reframe(its.sh, texture_eval(s, s.textures[sh.normal_map - 1], its.u, its.v));
        return;
    }
    // mesh.cpp:141-196
    float bx = 1 - (its.u + its.v), by = its.u, bz = its.v;
    V3 p0, p1, p2;
    uint32_t vi[3];
    tri_verts(s, sh, prim, p0, p1, p2, vi);
    its.p = bx * p0 + by * p1 + bz * p2;
    if (sh.has_uvs) {
        const float *u0 = &s.UV[2 * vi[0]], *u1 = &s.UV[2 * vi[1]], *u2 = &s.UV[2 * vi[2]];
        its.u = bx * u0[0] + by * u1[0] + bz * u2[0];
        its.v = bx * u0[1] + by * u1[1] + bz * u2[1];
    }
    its.geo = Frame::from_n(normalized(cross(p1 - p0, p2 - p0)));
    if (sh.has_normals) {
        V3 nrm = normalized(bx * s.N[vi[0]] + by * s.N[vi[1]] + bz * s.N[vi[2]]);
        if (sh.has_uvs) {
            V3 tg = normalized(bx * s.T[vi[0]] + by * s.T[vi[1]] + bz * s.T[vi[2]]);
            V3 bt = normalized(bx * s.BT[vi[0]] + by * s.BT[vi[1]] + bz * s.BT[vi[2]]);
            if (sh.normal_map)  // mesh.cpp:173-183
                nrm = tbn_normal(tg, bt, nrm, texture_eval(s, s.textures[sh.normal_map - 1], its.u, its.v));
            its.sh.s = tg;
            its.sh.t = bt;
            its.sh.n = nrm;
        } else {
            its.sh = Frame::from_n(nrm);
        }
    } else {
        its.sh = its.geo;
    }
}

// BoundingBox::rayIntersect (bbox.h:336-363)
bool box_intersect(const float *mn, const float *mx, const Ray &ray) {
    float near_t = -std::numeric_limits<float>::infinity();
    float far_t = std::numeric_limits<float>::infinity();
    const float o[3] = {ray.o.x, ray.o.y, ray.o.z}, d[3] = {ray.d.x, ray.d.y, ray.d.z},
                r[3] = {ray.drcp.x, ray.drcp.y, ray.drcp.z};
    for (int i = 0; i < 3; i++) {
        float origin = o[i], min_v = mn[i], max_v = mx[i];
        if (d[i] == 0) {
            if (origin < min_v || origin > max_v) return false;
        } else {
            float t1 = (min_v - origin) * r[i];
            float t2 = (max_v - origin) * r[i];
            if (t1 > t2) std::swap(t1, t2);
            near_t = std::max(t1, near_t);
            far_t = std::min(t2, far_t);
            if (!(near_t <= far_t)) return false;
        }
    }
    return ray.mint <= far_t && near_t <= ray.maxt;
}

// BVH::rayIntersect (bvh.cpp:402-460)
bool bvh_intersect(const no_scene &s, const Ray &_ray, Its &its, bool shadow, uint32_t *out_prim = nullptr,
                   float *out_bary = nullptr) {
    uint32_t node_idx = 0, stack_idx = 0, stack[64];
    its.t = std::numeric_limits<float>::infinity();
    Ray ray(_ray);
    if (ray.mint == kEps) {
        float m = std::max(std::max(std::fabs(ray.o.x), std::fabs(ray.o.y)), std::fabs(ray.o.z));
        ray.mint = std::max(ray.mint, ray.mint * m);
    }
    if (s.nodes.empty() || ray.maxt < ray.mint) return false;
    bool found = false;
    uint32_t f = 0, fshape = 0;
    float hu = 0, hv = 0;
    while (true) {
        const BNode &node = s.nodes[node_idx];
        if (!box_intersect(node.mn, node.mx, ray)) {
            if (stack_idx == 0) break;
            node_idx = stack[--stack_idx];
            continue;
        }
        if (!node.leaf()) {
            stack[stack_idx++] = node.w1;
            node_idx++;
        } else {
            for (uint32_t i = node.w1, end = node.w1 + node.size(); i < end; ++i) {
                uint32_t idx = s.indices[i];
                uint32_t sh = find_shape(s, idx);
                float u = 0, v = 0, t = 0;
                bool hit = s.shapes[sh].type == NH_SHAPE_MESH ? mesh_intersect(s, s.shapes[sh], idx, ray, u, v, t)
                                                             : sphere_intersect(s.shapes[sh], ray, t);
                if (hit) {
                    if (shadow) return true;
                    found = true;
                    ray.maxt = its.t = t;
                    hu = u;
                    hv = v;
                    f = idx;
                    fshape = sh;
                }
            }
            if (stack_idx == 0) break;
            node_idx = stack[--stack_idx];
        }
    }
    if (found) {
        its.u = hu;
        its.v = hv;
        if (out_prim) *out_prim = s.shape_offset[fshape] + f;
        if (out_bary) { out_bary[0] = hu; out_bary[1] = hv; }
        set_hit_information(s, fshape, f, ray, its);
    }
    return found;
}

// ---- emitters (src/emitters/arealight.cpp, pointlight.cpp) ---------------
struct ERec {  // EmitterQueryRecord (emitter.h)
    V3 ref = mk(0, 0, 0), p = mk(0, 0, 0), n = mk(0, 0, 0), wi = mk(0, 0, 0);
    float pdf = 0;
    Ray shadow;
};
inline ERec erec(V3 ref, V3 p, V3 n) {
    ERec r;
    r.ref = ref;
    r.p = p;
    r.n = n;
    r.wi = normalized(p - ref);
    return r;
}


// ---- EnvMap (environmentmap.cpp:73-169) + PNGTexture::eval (PNGTexture.cpp:125-160) ----------
// M_PI is Nori's float constant (common.h:61): every angle expression is fp32.
V3 spherical_direction(float theta, float phi) {  // common.cpp:270-281 (sincosf)
    float st = f_sin(theta), ct = f_cos(theta), sp = f_sin(phi), cp = f_cos(phi);
    return mk(st * cp, st * sp, ct);
}
void spherical_coordinates(V3 v, float &theta, float &phi) {  // common.cpp:283-291
    theta = f_acos(v.z);
    phi = f_atan2(v.y, v.x);
    if (phi < 0) phi += 2 * kPi;
}
// the texel lookup of PNGTexture::eval (PNGTexture.cpp:147-155), written as the reference writes it: the float ->
// unsigned casts are compiled by g++ for x86-64 (cvttss2si to 64 bits, low word: trunc(x) mod 2^32 for
// |x| < 2^63, else 0), which is what the reference binary executes for negative or huge products
V3 png_lookup(const float *d, unsigned width, unsigned height, float scale_u, float scale_v, float u, float v) {
    unsigned int w = static_cast<unsigned int>((u) * scale_u * (float)width);
    unsigned int h = height - static_cast<unsigned int>((v) * scale_v * (float)height);
    unsigned int index = (h * width + w) % (width * height);
    return mk(d[4 * (size_t)index], d[4 * (size_t)index + 1], d[4 * (size_t)index + 2]);
}

// Matrix3f * Vector3f in Eigen 3.3.8's order (x0*y0 + (x1*y1 + x2*y2) per row; m row-major)
inline V3 rot3(const float *m, V3 w) {
    return mk(m[0] * w.x + (m[1] * w.y + m[2] * w.z), m[3] * w.x + (m[4] * w.y + m[5] * w.z),
              m[6] * w.x + (m[7] * w.y + m[8] * w.z));
}

V3 env_tex_eval(const no_scene &s, float u, float v) {
    const float *d = s.env_rgba.data();
    if (s.env.constant) return mk(d[0], d[1], d[2]);  // ConstantTexture::eval
    if (s.env.spherical) {
        // rot * wi: Eigen's Matrix3f * Vector3f (PNGTexture.cpp:133-140; identity for eulerAngles = 0)
        const V3 wi = rot3(s.env.rotation, spherical_direction(v * kPi, u * 2.f * kPi));
        float th, ph;
        spherical_coordinates(wi, th, ph);
        u = ph / (2.f * kPi);
        v = th / kPi;
    } else {
        u += s.env.offset_u;
        v += s.env.offset_v;
    }
    return png_lookup(d, (unsigned)s.env.width, (unsigned)s.env.height, s.env.scale_u, s.env.scale_v, u, v);
}
V3 env_eval(const no_scene &s, V3 wi) {  // EnvMap::eval
    float th, ph;
    spherical_coordinates(wi, th, ph);
    const float u = ph / (2.f * kPi), v = th / kPi;
    return cmul(env_tex_eval(s, u, v), mk(s.env.radiance[0], s.env.radiance[1], s.env.radiance[2]));
}
float env_pdf(const no_scene &s, V3 wi) {  // EnvMap::pdf
    const float sphere_pdf = 0.25f / kPi;  // squareToUniformSpherePdf((1,0,0))
    if (s.env.width == 1 && s.env.height == 1) return sphere_pdf;
    return luminance(env_eval(s, wi)) * s.env.normalization / sphere_pdf * (float)(unsigned)s.env.height *
           (float)(unsigned)s.env.width;
}

// Texture<Color3f>::eval of a BSDF albedo (src/textures/consttexture.cpp, checkerboard.cpp:29-47,
// PNGTexture.cpp:125-160)
V3 texture_eval(const no_scene &s, const nh_texture &t, float u, float v) {
    if (t.type == NH_TEXTURE_CHECKERBOARD) {
        float ox = u / t.scale[0] - t.delta[0];
        float oy = v / t.scale[1] - t.delta[1];
        // int(float) as the x86-64 reference executes it (cvttss2si: NaN / out of range -> INT_MIN)
        int x = int(ox) + (ox < 0.f);
        int y = int(oy) + (oy < 0.f);
        // (x + y) % 2 == 0 with the reference's wrap-around int addition
        if ((int)((unsigned)x + (unsigned)y) % 2 == 0) return mk(t.value1[0], t.value1[1], t.value1[2]);
        return mk(t.value2[0], t.value2[1], t.value2[2]);
    }
    if (t.type == NH_TEXTURE_PNG) {
        if (t.spherical) {
            const V3 wi = rot3(t.rotation, spherical_direction(v * kPi, u * 2.f * kPi));
            float th, ph;
            spherical_coordinates(wi, th, ph);
            u = ph / (2.f * kPi);
            v = th / kPi;
        } else {
            u += t.offset_u;
            v += t.offset_v;
        }
        V3 out = png_lookup(s.texels.data() + 4 * (size_t)t.texel_offset, (unsigned)t.width, (unsigned)t.height,
                            t.scale_u, t.scale_v, u, v);
        return t.linear ? normal_blend(out, t.intensity) : out;  // !sRgb: a normal map
    }
    return mk(t.value1[0], t.value1[1], t.value1[2]);
}

V3 diffuse_albedo(const nh_bsdf &b, const BRec &r) {
    if (b.albedo_texture == 0 || !r.scene) return mk(b.albedo[0], b.albedo[1], b.albedo[2]);
    return texture_eval(*r.scene, r.scene->textures[b.albedo_texture - 1], r.u, r.v);
}
// bRec.uv = its.uv
inline void set_uv(BRec &r, const no_scene &s, const Its &its) {
    r.u = its.u;
    r.v = its.v;
    r.scene = &s;
}

size_t dpdf_sample(const float *cdf, size_t n_cdf, float x) {  // dpdf.h:124-130
    const float *e = std::lower_bound(cdf, cdf + n_cdf, x);
    size_t index = (size_t)std::max((ptrdiff_t)0, (e - cdf) - 1);
    return std::min(index, n_cdf - 2);
}

V3 emitter_eval(const no_scene &s, const nh_emitter &e, const ERec &r) {
    if (e.type == NH_EMITTER_AREA) {  // arealight.cpp:58-72
        if (dot(r.n, -r.wi) < 0.f) return mk(0, 0, 0);
        return mk(e.radiance[0], e.radiance[1], e.radiance[2]);
    }
    if (e.type == NH_EMITTER_POINT) {  // pointlight.cpp:70-76
        V3 pos = mk(e.position[0], e.position[1], e.position[2]);
        return mk(e.radiance[0], e.radiance[1], e.radiance[2]) / sqnorm(r.ref - pos);
    }
    (void)s;
    return mk(0, 0, 0);
}
float emitter_pdf(const no_scene &s, const nh_emitter &e, const ERec &r) {
    if (e.type == NH_EMITTER_ENVMAP) return env_pdf(s, r.wi);
    if (e.type == NH_EMITTER_AREA) {  // arealight.cpp:107-125
        if (dot(r.n, -r.wi) < 0.f) return 0.f;
        float prob = s.shapes[e.shape].type == NH_SHAPE_MESH
                         ? s.shapes[e.shape].pdf_normalization
                         : (float)(std::pow(1.f / s.shapes[e.shape].radius, 2) * (double)(0.25f / kPi));
        return prob * sqnorm(r.p - r.ref) / std::fabs(dot(r.n, -r.wi));
    }
    return 1.f;  // point light
}
V3 emitter_sample(const no_scene &s, const nh_emitter &e, ERec &r, float sx, float sy) {
    if (e.type == NH_EMITTER_ENVMAP) {  // EnvMap::sample (environmentmap.cpp:73-101)
        const unsigned W = (unsigned)s.env.width, H = (unsigned)s.env.height;
        const size_t elem = dpdf_sample(s.env_cdf.data(), s.env_cdf.size(), sx);
        const float i = (int)(elem / W) / (float)H, j = (int)(elem % W) / (float)W;
        V3 v = (W == 1 && H == 1) ? square_to_uniform_sphere(sx, sy) : spherical_direction(j * kPi, i * 2.0f * kPi);
        V3 v_inf = mk(v.x * 1.f / kEps, v.y * 1.f / kEps, v.z * 1.f / kEps);
        r.n = -v;
        r.p = v_inf;
        r.wi = normalized(r.p - r.ref);
        r.shadow = make_ray(r.p, -r.wi, kEps, norm(r.p - r.ref) - kEps);
        r.pdf = env_pdf(s, r.wi);
        if (r.pdf < kEps) return mk(0, 0, 0);
        return env_eval(s, r.wi) / r.pdf;
    }
    if (e.type == NH_EMITTER_POINT) {  // pointlight.cpp:47-66
        V3 pos = mk(e.position[0], e.position[1], e.position[2]);
        r.shadow = make_ray(pos, normalized(r.ref - pos), kEps, norm(r.ref - pos) - kEps);
        r.wi = normalized(pos - r.ref);
        r.pdf = 1.f;
        return emitter_eval(s, e, r) / 1.f;
    }
    // AreaEmitter::sample (arealight.cpp:75-104) -> Shape::sampleSurface
    const nh_shape &sh = s.shapes[e.shape];
    V3 p, n;
    if (sh.type == NH_SHAPE_MESH) {  // mesh.cpp:50-71
        const float *cdf = &s.area_cdf[sh.pdf_offset];
        size_t idt = dpdf_sample(cdf, (size_t)sh.n_faces + 1, sx);
        sx = (sx - cdf[idt]) / (cdf[idt + 1] - cdf[idt]);
        V3 bc = square_to_uniform_triangle(sx, sy);
        V3 p0, p1, p2;
        uint32_t vi[3];
        tri_verts(s, sh, (uint32_t)idt, p0, p1, p2, vi);
        p = bc.x * p0 + bc.y * p1 + bc.z * p2;
        if (sh.has_normals)
            n = normalized(bc.x * s.N[vi[0]] + bc.y * s.N[vi[1]] + bc.z * s.N[vi[2]]);
        else
            n = normalized(cross(p1 - p0, p2 - p0));
    } else {  // sphere.cpp:126-131
        V3 q = square_to_uniform_sphere(sx, sy);
        p = mk(sh.center[0], sh.center[1], sh.center[2]) + sh.radius * q;
        n = q;
    }
    V3 ref = r.ref;
    r = erec(ref, p, n);
    r.shadow = make_ray(r.p, -r.wi, kEps, norm(r.p - r.ref) - kEps);
    float probs = emitter_pdf(s, e, r);
    r.pdf = probs;
    if (std::fabs(probs) < kEps) return mk(0, 0, 0);
    return emitter_eval(s, e, r) / probs;
}

// ---- integrators ----------------------------------------------------------
V3 li_path_mis(const no_scene &s, Sampler &smp, const Ray &ray) {  // path_mis.cpp:16-150
    V3 li = mk(0, 0, 0), t = mk(1, 1, 1);
    Ray trace = ray;
    float w_mats = 1.f, w_ems = 0.f;
    const float n_lights = (float)s.emitters.size();
    while (true) {
        V3 li_ems = mk(0, 0, 0);
        float pdfems = 0.f, pdfmat = 0.f, pdfems_mats = 0.f, pdfmat_ems = 0.f;
        Its its;
        if (!bvh_intersect(s, trace, its, false)) {
            if (s.envmap >= 0) li = li + cmul(t, env_eval(s, trace.d));  // path_mis.cpp:32-43
            break;
        }
        const nh_shape &shape = s.shapes[its.shape];
        const nh_bsdf &bsdf = s.bsdfs[shape.bsdf];
        if (shape.emitter >= 0) {
            ERec eqr = erec(trace.o, its.p, its.sh.n);
            V3 e = emitter_eval(s, s.emitters[shape.emitter], eqr);
            li = li + cmul(w_mats * t, e);
        }
        float succ = std::min(max_coeff(t), 0.99f);
        succ = std::max(succ, kEps);
        if (smp.next1d() > succ) break;
        t = t / succ;

        size_t ei = dpdf_sample(s.emitter_cdf.data(), s.emitter_cdf.size(), smp.next1d());
        const nh_emitter &em = s.emitters[ei];
        ERec eqr_ems;
        eqr_ems.ref = its.p;
        float ex, ey;
        smp.next2d(ex, ey);
        V3 ems_col = emitter_sample(s, em, eqr_ems, ex, ey);
        V3 we = its.sh.to_local(eqr_ems.wi);
        if (!is_zero(ems_col)) {
            Its dummy;
            if (!bvh_intersect(s, eqr_ems.shadow, dummy, true)) {
                BRec bq;
                set_uv(bq, s, its);
                bq.wi = its.sh.to_local(-trace.d);
                bq.wo = we;
                bq.measure = ESolidAngle;
                V3 f = bsdf_eval(bsdf, bq);
                float cs = we.z;
                li_ems = cmul(ems_col * cs, f) * n_lights;
                pdfems_mats = bsdf_pdf(bsdf, bq);
                pdfems = emitter_pdf(s, em, eqr_ems) / n_lights;
            }
        }
        if ((pdfems_mats + pdfems) > kEps) w_ems = pdfems / (pdfems_mats + pdfems);

        BRec br;
        set_uv(br, s, its);
        br.wi = its.sh.to_local(-trace.d);
        float bx, by;
        smp.next2d(bx, by);
        V3 bsdf_col = bsdf_sample(bsdf, br, bx, by);
        if (!is_zero(bsdf_col)) {
            Ray probe = make_ray(its.p, its.sh.to_world(br.wo));
            Its its_s;
            if (bvh_intersect(s, probe, its_s, false)) {
                const nh_shape &hs = s.shapes[its_s.shape];
                if (hs.emitter >= 0) {
                    ERec eqr_mats = erec(its.p, its_s.p, its_s.sh.n);
                    pdfmat = bsdf_pdf(bsdf, br);
                    pdfmat_ems = emitter_pdf(s, s.emitters[hs.emitter], eqr_mats) / n_lights;
                    if ((pdfmat + pdfmat_ems) > kEps) w_mats = pdfmat / (pdfmat + pdfmat_ems);
                }
            }
        }
        if (br.measure == EDiscrete) {
            w_ems = 0.f;
            w_mats = 1.f;
        }
        li = li + cmul(w_ems * t, li_ems);
        t = cmul(t, bsdf_col);
        trace = make_ray(its.p, its.sh.to_world(br.wo));
    }
    return li;
}

V3 li_path_mats(const no_scene &s, Sampler &smp, const Ray &ray) {  // path_mats.cpp:16-78
    V3 li = mk(0, 0, 0), t = mk(1, 1, 1);
    Ray trace = ray;
    int counter = 0;
    while (true) {
        Its its;
        if (!bvh_intersect(s, trace, its, false)) {
            if (s.envmap >= 0) li = li + cmul(t, env_eval(s, trace.d));  // path_mats.cpp:26-35
            break;
        }
        const nh_shape &shape = s.shapes[its.shape];
        const nh_bsdf &bsdf = s.bsdfs[shape.bsdf];
        if (shape.emitter >= 0) {
            ERec eqr = erec(trace.o, its.p, its.sh.n);
            li = li + cmul(t, emitter_eval(s, s.emitters[shape.emitter], eqr));
        }
        float succ = std::min(max_coeff(t), 0.99f);
        if (counter < 3) counter++;
        else if (smp.next1d() > succ) break;
        else t = t / succ;
        BRec br;
        set_uv(br, s, its);
        br.wi = its.sh.to_local(-trace.d);
        br.measure = ESolidAngle;
        float bx, by;
        smp.next2d(bx, by);
        V3 col = bsdf_sample(bsdf, br, bx, by);
        t = cmul(t, col);
        trace = make_ray(its.p, its.sh.to_world(br.wo));
    }
    return li;
}


// ---- single-bounce direct integrators ------------------------------------
// first hit of the camera ray: miss -> environment (direct_*.cpp:17-26), emitter hit -> its radiance
static bool direct_first_hit(const no_scene &s, const Ray &ray, Its &its, V3 &result) {
    if (!bvh_intersect(s, ray, its, false)) {
        result = s.envmap >= 0 ? env_eval(s, ray.d) : mk(0, 0, 0);
        return false;
    }
    result = mk(0, 0, 0);
    const nh_shape &shape = s.shapes[its.shape];
    if (shape.emitter >= 0) result = result + emitter_eval(s, s.emitters[shape.emitter], erec(ray.o, its.p, its.sh.n));
    return true;
}

V3 li_direct_ems(const no_scene &s, Sampler &smp, const Ray &ray) {  // direct_ems.cpp:14-70
    Its its;
    V3 result;
    if (!direct_first_hit(s, ray, its, result)) return result;
    const nh_bsdf &bsdf = s.bsdfs[s.shapes[its.shape].bsdf];
    const V3 wo = its.sh.to_local(-ray.d);
    for (const nh_emitter &l : s.emitters) {  // scene->getLights(), each with its own next2D
        ERec eqr;
        eqr.ref = its.p;
        float ex, ey;
        smp.next2d(ex, ey);
        V3 li = emitter_sample(s, l, eqr, ex, ey);
        if (is_zero(li)) continue;
        Its dummy;
        if (bvh_intersect(s, eqr.shadow, dummy, true)) continue;
        BRec bq;
        set_uv(bq, s, its);
        bq.wi = wo;
        bq.wo = its.sh.to_local(eqr.wi);
        bq.measure = ESolidAngle;
        V3 f = bsdf_eval(bsdf, bq);
        result = result + cmul(li * std::abs(its.sh.to_local(eqr.wi).z), f);
    }
    return result;
}

V3 li_direct_mats(const no_scene &s, Sampler &smp, const Ray &ray) {  // direct_mats.cpp:16-83
    Its its;
    V3 result;
    if (!direct_first_hit(s, ray, its, result)) return result;
    const nh_bsdf &bsdf = s.bsdfs[s.shapes[its.shape].bsdf];
    BRec br;
    set_uv(br, s, its);
    br.wi = its.sh.to_local(-ray.d);
    br.measure = ESolidAngle;
    float bx, by;
    smp.next2d(bx, by);
    V3 col = bsdf_sample(bsdf, br, bx, by);
    if (is_zero(col)) return result;
    Ray sec = make_ray(its.p, its.sh.to_world(br.wo));
    Its its2;
    if (!bvh_intersect(s, sec, its2, false)) {
        if (s.envmap >= 0) result = result + cmul(env_eval(s, sec.d), col);
        return result;
    }
    const nh_shape &hs = s.shapes[its2.shape];
    if (hs.emitter >= 0) result = result + cmul(emitter_eval(s, s.emitters[hs.emitter], erec(its.p, its2.p, its2.sh.n)), col);
    return result;
}

V3 li_direct_mis(const no_scene &s, Sampler &smp, const Ray &ray) {  // direct_mis.cpp:15-143
    Its its;
    V3 result;
    if (!direct_first_hit(s, ray, its, result)) return result;
    const nh_bsdf &bsdf = s.bsdfs[s.shapes[its.shape].bsdf];
    const float n_lights = (float)s.emitters.size();
    V3 result_ems = mk(0, 0, 0), result_mats = mk(0, 0, 0);
    float w_ems = 0.f, w_mat = 0.f;
    size_t ei = dpdf_sample(s.emitter_cdf.data(), s.emitter_cdf.size(), smp.next1d());
    const nh_emitter &l_ems = s.emitters[ei];
    ERec eqr;
    eqr.ref = its.p;
    float ex, ey;
    smp.next2d(ex, ey);
    V3 li = emitter_sample(s, l_ems, eqr, ex, ey);
    if (!is_zero(li)) {
        Its dummy;
        if (!bvh_intersect(s, eqr.shadow, dummy, true)) {
            BRec bq;
            set_uv(bq, s, its);
            bq.wi = its.sh.to_local(-ray.d);
            bq.wo = its.sh.to_local(eqr.wi);
            bq.measure = ESolidAngle;
            V3 f = bsdf_eval(bsdf, bq);
            float cs = its.sh.to_local(eqr.wi).z;
            float pdf_ems = emitter_pdf(s, l_ems, eqr) / n_lights;
            float pdf_mat = bsdf_pdf(bsdf, bq);
            result_ems = cmul(li * cs, f) * n_lights;
            if (pdf_ems + pdf_mat > kEps) w_ems = pdf_ems / (pdf_ems + pdf_mat);
        } else if (s.envmap >= 0) {
            result_ems = cmul(li, env_eval(s, eqr.shadow.d));
        }
    }
    BRec bm;
    set_uv(bm, s, its);
    bm.wi = its.sh.to_local(-ray.d);
    bm.measure = ESolidAngle;
    float bx, by;
    smp.next2d(bx, by);
    V3 col = bsdf_sample(bsdf, bm, bx, by);
    if (!is_zero(col)) {
        Ray sr = make_ray(its.p, its.sh.to_world(bm.wo));
        Its its2;
        if (bvh_intersect(s, sr, its2, false) && s.shapes[its2.shape].emitter >= 0) {
            const nh_emitter &e2 = s.emitters[s.shapes[its2.shape].emitter];
            ERec q2 = erec(its.p, its2.p, its2.sh.n);
            result_mats = cmul(col, emitter_eval(s, e2, q2));
            float pdf_mat = bsdf_pdf(bsdf, bm);
            float pdf_e = emitter_pdf(s, e2, q2) / n_lights;
            if (pdf_mat + pdf_e > kEps) w_mat = pdf_mat / (pdf_mat + pdf_e);
        } else if (s.envmap >= 0) {
            result_mats = cmul(col, env_eval(s, sr.d));
        }
    }
    return result + w_ems * result_ems + w_mat * result_mats;
}

// DirectIntegrator::Li (direct.cpp:17-63, the point-light integrator of scenes/pa1): every emitter is
// sampled once (its own next2D) and its shadow ray traced; unoccluded samples add
// li * |wi . n| / |wi| * f(wi = light, wo = toward the ray origin). No emitter-hit term.
V3 li_direct(const no_scene &s, Sampler &smp, const Ray &ray) {
    Its its;
    if (!bvh_intersect(s, ray, its, false)) return s.envmap >= 0 ? env_eval(s, ray.d) : mk(0, 0, 0);
    V3 result = mk(0, 0, 0);
    const nh_bsdf &bsdf = s.bsdfs[s.shapes[its.shape].bsdf];
    const V3 wo = its.sh.to_local(normalized(ray.o - its.p));
    for (const nh_emitter &l : s.emitters) {
        ERec rec;
        rec.ref = its.p;
        float ex, ey;
        smp.next2d(ex, ey);
        const V3 li = emitter_sample(s, l, rec, ex, ey);
        const V3 wi = its.sh.to_local(rec.wi);
        Its dummy;
        if (bvh_intersect(s, rec.shadow, dummy, true)) continue;
        BRec bq;
        set_uv(bq, s, its);
        bq.wi = wi;
        bq.wo = wo;
        bq.measure = ESolidAngle;
        const V3 f = bsdf_eval(bsdf, bq);
        const float cs = std::abs(dot(rec.wi, its.sh.n)) / norm(rec.wi);
        result = result + cmul(li * cs, f);
    }
    return result;
}

// NormalIntegrator::Li (normals.cpp:15-33): |shFrame.toWorld(direction)| at the first hit, the envmap on a miss
V3 li_normals(const no_scene &s, const Ray &ray) {
    Its its;
    if (!bvh_intersect(s, ray, its, false)) return s.envmap >= 0 ? env_eval(s, ray.d) : mk(0, 0, 0);
    const V3 n = its.sh.to_world(mk(s.normals_dir[0], s.normals_dir[1], s.normals_dir[2]));
    return mk(std::fabs(n.x), std::fabs(n.y), std::fabs(n.z));
}

inline bool has_dof(const nh_camera &c) { return c.lens_radius > kEps; }  // perspective.cpp:114

// PerspectiveCamera::sampleRay (perspective.cpp:97-141). lens: the two floats the static camera sampler returns
// for this ray (perspective.cpp:118-122), read only with depth of field.
Ray camera_ray(const nh_camera &c, float px, float py, const float *lens = nullptr) {
    const float *m = c.sample_to_camera;
    float in[4] = {px * c.inv_output_size[0], py * c.inv_output_size[1], 0.0f, 1.0f};
    float r[4];
    for (int i = 0; i < 4; ++i) {
        float acc = m[4 * i + 0] * in[0];
        acc = acc + m[4 * i + 1] * in[1];
        acc = acc + m[4 * i + 2] * in[2];
        acc = acc + m[4 * i + 3] * in[3];
        r[i] = acc;
    }
    V3 near_p = mk(r[0] / r[3], r[1] / r[3], r[2] / r[3]);
    const V3 d = normalized(near_p);
    V3 lo = mk(0.0f, 0.0f, 0.0f), ld = d;  // ray.o = Point3f(0, 0, 0), ray.d = d
    if (has_dof(c)) {
        float dx, dy;
        square_to_uniform_disk(lens[0], lens[1], dx, dy);
        const float plx = c.lens_radius * dx, ply = c.lens_radius * dy;  // m_lensRadius * Point2f
        const float ft = c.focal_distance / ld.z;
        const V3 pf = mk(lo.x + ft * ld.x, lo.y + ft * ld.y, lo.z + ft * ld.z);  // ray(ft) = o + t * d
        lo = mk(plx, ply, 0.f);
        ld = normalized(mk(pf.x - lo.x, pf.y - lo.y, pf.z - lo.z));
    }
    const float *w = c.camera_to_world;
    float o4[4];
    const float pin[4] = {lo.x, lo.y, lo.z, 1.0f};
    for (int i = 0; i < 4; ++i) {
        float acc = w[4 * i + 0] * pin[0];
        acc = acc + w[4 * i + 1] * pin[1];
        acc = acc + w[4 * i + 2] * pin[2];
        acc = acc + w[4 * i + 3] * pin[3];
        o4[i] = acc;
    }
    Ray ray;
    ray.o = mk(o4[0] / o4[3], o4[1] / o4[3], o4[2] / o4[3]);
    ray.d = mk(w[0] * ld.x + (w[1] * ld.y + w[2] * ld.z), w[4] * ld.x + (w[5] * ld.y + w[6] * ld.z),
               w[8] * ld.x + (w[9] * ld.y + w[10] * ld.z));
    float inv_z = 1.0f / d.z;  // the pinhole direction (perspective.cpp:135)
    ray.mint = c.near_clip * inv_z;
    ray.maxt = c.far_clip * inv_z;
    ray.drcp = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    return ray;
}

V3 li(const no_scene &s, Sampler &smp, const Ray &r) {
    switch (s.integrator) {
        case NH_INTEGRATOR_PATH_MATS: return li_path_mats(s, smp, r);
        case NH_INTEGRATOR_DIRECT_EMS: return li_direct_ems(s, smp, r);
        case NH_INTEGRATOR_DIRECT_MATS: return li_direct_mats(s, smp, r);
        case NH_INTEGRATOR_DIRECT_MIS: return li_direct_mis(s, smp, r);
        case NH_INTEGRATOR_DIRECT: return li_direct(s, smp, r);
        case NH_INTEGRATOR_NORMALS: return li_normals(s, r);
        default: return li_path_mis(s, smp, r);
    }
}

// ---- ImageBlock (src/utils/block.cpp) ------------------------------------
struct Block {
    int ox, oy, sx, sy, id;
    int cols, rows;  // 32 + 2*border
    std::vector<float> px;  // rgbw
};

// ImageBlock::put(pos, value) (block.cpp:93-123)
bool block_put(Block &b, const nh_filter &f, float spx, float spy, V3 v) {
    if (!is_valid(v)) return false;
    float pos_x = spx - 0.5f - (float)(b.ox - f.border);
    float pos_y = spy - 0.5f - (float)(b.oy - f.border);
    int x0 = (int)std::ceil(pos_x - f.radius), y0 = (int)std::ceil(pos_y - f.radius);
    int x1 = (int)std::floor(pos_x + f.radius), y1 = (int)std::floor(pos_y + f.radius);
    x0 = std::max(x0, 0); y0 = std::max(y0, 0);
    x1 = std::min(x1, b.cols - 1); y1 = std::min(y1, b.rows - 1);
    float wx[8], wy[8];
    for (int x = x0, i = 0; x <= x1; ++x) wx[i++] = f.table[(int)(std::fabs((float)x - pos_x) * f.lookup_factor)];
    for (int y = y0, i = 0; y <= y1; ++y) wy[i++] = f.table[(int)(std::fabs((float)y - pos_y) * f.lookup_factor)];
    for (int y = y0, yr = 0; y <= y1; ++y, ++yr)
        for (int x = x0, xr = 0; x <= x1; ++x, ++xr) {
            float *p = &b.px[4 * ((size_t)y * b.cols + x)];
            p[0] += v.x * wx[xr] * wy[yr];
            p[1] += v.y * wx[xr] * wy[yr];
            p[2] += v.z * wx[xr] * wy[yr];
            p[3] += 1.0f * wx[xr] * wy[yr];
        }
    return true;
}

// BlockGenerator spiral order (block.cpp:151-199)
std::vector<std::pair<int, int>> spiral_blocks(int w, int h, int bs) {
    int nbx = (int)std::ceil(w / (float)bs), nby = (int)std::ceil(h / (float)bs);
    std::vector<std::pair<int, int>> out;
    int left = nbx * nby;
    int dir = 0, bx = nbx / 2, by = nby / 2, steps_left = 1, num_steps = 1;
    while (left > 0) {
        out.emplace_back(bx, by);
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
    return out;
}

// Position of each pixel's camera ray within one sample round of the reference's serial render order: blocks in
// BlockGenerator order, edge blocks clipped (block.cpp:174-176), a block's pixels x-major
// (Independent::getSampleIndices, independent.cpp:85-99)
std::vector<uint32_t> serial_ray_index(int w, int h, int bs) {
    std::vector<uint32_t> idx((size_t)w * h);
    uint32_t k = 0;
    for (auto &b : spiral_blocks(w, h, bs)) {
        const int ox = b.first * bs, oy = b.second * bs, sx = std::min(bs, w - ox), sy = std::min(bs, h - oy);
        for (int x = 0; x < sx; ++x)
            for (int y = 0; y < sy; ++y) idx[(size_t)(oy + y) * w + (ox + x)] = k++;
    }
    return idx;
}

// The lens sample of serial camera ray k (perspective.cpp:118-122): the camera's static Independent sampler is a
// default-state pcg32 that is never prepared (pcg32.h:40), two floats per sampleRay call, so ray k reads draws
// 2k and 2k + 1 -- pcg32::advance gets there without the k - 1 rays before it. Point2f(nextFloat(), nextFloat()) takes them as
// (x, y) = (2k + 1, 2k) when the compiler evaluates the arguments right to left (g++: nh_camera.lens_draw_order
// NH_LENS_DRAWS_RTL), (2k, 2k + 1) left to right (clang)
void lens_jump(const nh_camera &c, uint64_t k, float out[2]) {
    Pcg32 r;
    r.advance((int64_t)(2 * k));
    const float a = r.next_float(), b = r.next_float();
    out[0] = c.lens_draw_order == NH_LENS_DRAWS_RTL ? b : a;
    out[1] = c.lens_draw_order == NH_LENS_DRAWS_RTL ? a : b;
}

}  // namespace

extern "C" {

int no_env_cdf(const no_scene *s, const float **cdf, uint32_t *n, float *normalization) {
    if (!s || s->envmap < 0) return NH_ERR_INVALID;
    *cdf = s->env_cdf.data();
    *n = (uint32_t)s->env_cdf.size();
    *normalization = s->env.normalization;
    return NH_OK;
}

int no_scene_create(const nh_scene_desc *d, no_scene **out) {
    if (!d || !out) return NH_ERR_INVALID;
    auto s = std::make_unique<no_scene>();
    s->cam = d->camera;
    s->filter = d->filter;
    s->integrator = d->integrator;
    for (int i = 0; i < 3; ++i) s->normals_dir[i] = d->normals_direction[i];
    s->shapes.assign(d->shapes, d->shapes + d->n_shapes);
    s->bsdfs.assign(d->bsdfs, d->bsdfs + d->n_bsdfs);
    if (d->n_textures) s->textures.assign(d->textures, d->textures + d->n_textures);
    if (d->n_texels) s->texels.assign(d->texels, d->texels + 4 * (size_t)d->n_texels);
    for (const nh_bsdf &b : s->bsdfs)
        if (b.albedo_texture > s->textures.size()) return NH_ERR_INVALID;
    for (const nh_shape &sh : s->shapes)
        if (sh.normal_map > s->textures.size()) return NH_ERR_INVALID;
    s->emitters.assign(d->emitters, d->emitters + d->n_emitters);
    s->emitter_cdf.assign(d->emitter_cdf, d->emitter_cdf + d->n_emitters + 1);
    for (uint32_t i = 0; i < d->n_vertices; ++i) {
        s->V.push_back(mk(d->V[3 * i], d->V[3 * i + 1], d->V[3 * i + 2]));
        s->N.push_back(mk(d->N[3 * i], d->N[3 * i + 1], d->N[3 * i + 2]));
        s->T.push_back(mk(d->T[3 * i], d->T[3 * i + 1], d->T[3 * i + 2]));
        s->BT.push_back(mk(d->BT[3 * i], d->BT[3 * i + 1], d->BT[3 * i + 2]));
    }
    s->UV.assign(d->UV, d->UV + 2 * (size_t)d->n_vertices);
    s->F.assign(d->F, d->F + 3 * (size_t)d->n_faces);
    s->area_cdf.assign(d->area_cdf, d->area_cdf + d->n_area_cdf);
    s->envmap = d->envmap;
    if (d->envmap >= 0) {
        s->env = d->env;
        s->env_rgba.assign(d->env.rgba, d->env.rgba + 4 * (size_t)d->env.width * d->env.height);
        s->env.rgba = nullptr;
        s->env.cdf = nullptr;
        // EnvMap::calculateProbs (environmentmap.cpp:155-169) + DiscretePDF append/normalize
        // (dpdf.h:48-115), restated: texture evaluated at (row / H, col / W)
        const unsigned W = (unsigned)d->env.width, H = (unsigned)d->env.height;
        s->env_cdf.assign(1, 0.0f);
        for (unsigned i = 0; i < H; ++i)
            for (unsigned j = 0; j < W; ++j)
                s->env_cdf.push_back(s->env_cdf.back() + std::fabs(luminance(env_tex_eval(*s, i / (float)H, j / (float)W))));
        const float sum = s->env_cdf.back();
        if (sum > 0) {
            s->env.normalization = 1.0f / sum;
            for (size_t i = 1; i < s->env_cdf.size(); ++i) s->env_cdf[i] *= s->env.normalization;
            s->env_cdf.back() = 1.0f;
        } else {
            s->env.normalization = 0.0f;
        }
    }

    // ---- BVH::addShape / BVH::build, serial restatement (bvh.cpp:236-380) ----
    s->shape_offset.push_back(0u);
    for (int i = 0; i < 3; ++i) { s->bmin[i] = INFINITY; s->bmax[i] = -INFINITY; }
    for (auto &sh : s->shapes) {
        s->shape_offset.push_back(s->shape_offset.back() + (sh.type == NH_SHAPE_MESH ? sh.n_faces : 1u));
        for (int i = 0; i < 3; ++i) {
            s->bmin[i] = std::min(s->bmin[i], sh.bbox_min[i]);
            s->bmax[i] = std::max(s->bmax[i], sh.bbox_max[i]);
        }
    }
    const uint32_t size = s->shape_offset.back();
    if (size > 0) {
        no_scene &S = *s;
        struct Box {
            float mn[3], mx[3];
            void reset() { for (int i = 0; i < 3; ++i) { mn[i] = INFINITY; mx[i] = -INFINITY; } }
            void expand(const Box &b) {
                for (int i = 0; i < 3; ++i) { mn[i] = std::min(mn[i], b.mn[i]); mx[i] = std::max(mx[i], b.mx[i]); }
            }
            float area() const {
                float dd[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
                float result = 0.0f;
                for (int i = 0; i < 3; ++i) {
                    float term = 1.0f;
                    for (int j = 0; j < 3; ++j) if (i != j) term *= dd[j];
                    result += term;
                }
                return 2.0f * result;
            }
        };
        auto prim_box = [&S](uint32_t g) {
            uint32_t idx = g;
            uint32_t sh = find_shape(S, idx);
            const nh_shape &shp = S.shapes[sh];
            Box b;
            if (shp.type == NH_SHAPE_SPHERE) {
                for (int i = 0; i < 3; ++i) { b.mn[i] = shp.bbox_min[i]; b.mx[i] = shp.bbox_max[i]; }
                return b;
            }
            V3 p0, p1, p2;
            tri_verts(S, shp, idx, p0, p1, p2);
            float a[3] = {p0.x, p0.y, p0.z};
            for (int i = 0; i < 3; ++i) b.mn[i] = b.mx[i] = a[i];
            for (V3 p : {p1, p2}) {
                float q[3] = {p.x, p.y, p.z};
                for (int i = 0; i < 3; ++i) { b.mn[i] = std::min(b.mn[i], q[i]); b.mx[i] = std::max(b.mx[i], q[i]); }
            }
            return b;
        };
        auto centroid = [&S](uint32_t g, int axis) {
            uint32_t idx = g;
            uint32_t sh = find_shape(S, idx);
            const nh_shape &shp = S.shapes[sh];
            if (shp.type == NH_SHAPE_SPHERE) return shp.center[axis];
            V3 p0, p1, p2;
            tri_verts(S, shp, idx, p0, p1, p2);
            V3 c = (1.0f / 3.0f) * (p0 + p1 + p2);
            return axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
        };
        struct Node { uint32_t w0, w1; Box box; };
        std::vector<Node> nodes(2 * (size_t)size);
        for (auto &n : nodes) { n.w0 = n.w1 = 0; for (int i = 0; i < 3; ++i) n.box.mn[i] = n.box.mx[i] = 0.f; }
        for (int i = 0; i < 3; ++i) { nodes[0].box.mn[i] = s->bmin[i]; nodes[0].box.mx[i] = s->bmax[i]; }
        s->indices.resize(size);
        for (uint32_t i = 0; i < size; ++i) s->indices[i] = i;
        std::vector<uint32_t> temp(size);
        uint32_t *base = s->indices.data();

        // Test-speed only: the centroid and box of every primitive are computed once (the same
        // float values the reference recomputes inside each comparison, so every sort sees the same
        // comparison results and produces the same order), and large disjoint subtrees are built
        // on their own threads (they own disjoint node slots, index ranges and scratch).
        std::vector<float> cen[3];
        std::vector<Box> pbox(size);
        for (int a = 0; a < 3; ++a) cen[a].resize(size);
        for (uint32_t g = 0; g < size; ++g) {
            for (int a = 0; a < 3; ++a) cen[a][g] = centroid(g, a);
            pbox[g] = prim_box(g);
        }
        constexpr uint32_t kParallelPrims = 65536;
        const int max_threads = (int)std::max(1u, std::thread::hardware_concurrency());
        std::atomic<int> live_threads{1};
        // run a(); b(); -- a on another thread when the range is large and a thread is free
        auto fork2 = [&](uint32_t sz, const std::function<void()> &a, const std::function<void()> &b) {
            if (sz >= kParallelPrims && live_threads.fetch_add(1) < max_threads) {
                std::thread t(a);
                b();
                t.join();
                live_threads.fetch_sub(1);
            } else {
                if (sz >= kParallelPrims) live_threads.fetch_sub(1);
                a();
                b();
            }
        };
        std::function<void(uint32_t, uint32_t *, uint32_t *, uint32_t *)> serial;
        serial = [&](uint32_t node_idx, uint32_t *start, uint32_t *end, uint32_t *tmp) {
            Node &node = nodes[node_idx];
            uint32_t sz = (uint32_t)(end - start);
            float best_cost = (float)1 * sz;
            int64_t best_index = -1, best_axis = -1;
            float *left_areas = (float *)tmp;
            for (int axis = 0; axis < 3; ++axis) {
                const float *c = cen[axis].data();
                std::sort(start, end, [c](uint32_t f1, uint32_t f2) { return c[f1] < c[f2]; });
                Box bbox; bbox.reset();
                for (uint32_t i = 0; i < sz; ++i) { bbox.expand(pbox[start[i]]); left_areas[i] = (float)bbox.area(); }
                if (axis == 0) node.box = bbox;
                bbox.reset();
                float tri_factor = 1 / node.box.area();
                for (uint32_t i = sz - 1; i >= 1; --i) {
                    bbox.expand(pbox[start[i]]);
                    float la = left_areas[i - 1], ra = bbox.area();
                    uint32_t pl = i, pr = sz - i;
                    float cost = 2.0f * 1 + tri_factor * (pl * la + pr * ra);
                    if (cost < best_cost) { best_cost = cost; best_index = i; best_axis = axis; }
                }
            }
            if (best_index == -1) { node.w0 = 1u | (sz << 1); node.w1 = (uint32_t)(start - base); return; }
            const float *c = cen[best_axis].data();
            std::sort(start, end, [c](uint32_t f1, uint32_t f2) { return c[f1] < c[f2]; });
            uint32_t lc = (uint32_t)best_index, li = node_idx + 1, ri = node_idx + 2 * lc;
            node.w0 = 0u | ((uint32_t)best_axis << 1);
            node.w1 = ri;
            fork2(sz, [&, li, start, lc, tmp] { serial(li, start, start + lc, tmp); },
                  [&, ri, start, lc, end, tmp] { serial(ri, start + lc, end, tmp + lc); });
        };
        auto to_int = [](float x) -> int { if (!(x > -2147483904.0f && x < 2147483648.0f)) return INT32_MIN; return (int)x; };
        std::function<void(uint32_t, uint32_t *, uint32_t *, uint32_t *)> task;
        task = [&](uint32_t node_idx, uint32_t *start, uint32_t *end, uint32_t *tmp) {
            uint32_t sz = (uint32_t)(end - start);
            Node &node = nodes[node_idx];
            if (sz < 32) { serial(node_idx, start, end, tmp); return; }
            float e0 = node.box.mx[0] - node.box.mn[0], e1 = node.box.mx[1] - node.box.mn[1], e2 = node.box.mx[2] - node.box.mn[2];
            int axis = (e0 >= e1 && e0 >= e2) ? 0 : ((e1 >= e0 && e1 >= e2) ? 1 : 2);
            float mn = node.box.mn[axis], mx = node.box.mx[axis], inv = 16 / (mx - mn);
            uint32_t counts[16] = {0};
            Box bb[16];
            for (auto &b : bb) b.reset();
            for (uint32_t i = 0; i < sz; ++i) {
                uint32_t f = start[i];
                int index = std::min(std::max(to_int((cen[axis][f] - mn) * inv), 0), 15);
                counts[index]++;
                bb[index].expand(pbox[f]);
            }
            Box bl[16];
            bl[0] = bb[0];
            for (int i = 1; i < 16; ++i) { counts[i] += counts[i - 1]; bl[i] = bl[i - 1]; bl[i].expand(bb[i]); }
            Box br = bb[15], best_br;
            best_br.reset();
            int64_t best_index = -1;
            float best_cost = (float)1 * sz, tri_factor = (float)1 / node.box.area();
            for (int i = 14; i >= 0; --i) {
                uint32_t pl = counts[i], pr = sz - counts[i];
                float cost = 2.0f * 1 + tri_factor * (pl * bl[i].area() + pr * br.area());
                if (cost < best_cost) { best_cost = cost; best_index = i; best_br = br; }
                br.expand(bb[i]);
            }
            if (best_index == -1) { serial(node_idx, start, end, tmp); return; }
            uint32_t lc = counts[best_index], li = node_idx + 1, ri = node_idx + 2 * lc;
            nodes[li].box = bl[best_index];
            nodes[ri].box = best_br;
            node.w0 = 0u | ((uint32_t)axis << 1);
            node.w1 = ri;
            uint32_t il = 0, ir = lc;
            for (uint32_t i = 0; i < sz; ++i) {
                uint32_t f = start[i];
                int index = to_int((cen[axis][f] - mn) * inv);
                if (index <= best_index) tmp[il++] = f; else tmp[ir++] = f;
            }
            std::memcpy(start, tmp, sz * sizeof(uint32_t));
            fork2(sz, [&, li, start, lc, tmp] { task(li, start, start + lc, tmp); },
                  [&, ri, start, lc, end, tmp] { task(ri, start + lc, end, tmp + lc); });
        };
        task(0u, base, base + size, temp.data());
        // statistics + compaction (bvh.cpp:354-379)
        std::function<uint32_t(uint32_t)> count = [&](uint32_t i) -> uint32_t {
            if (nodes[i].w0 & 1u) return 1u;
            return count(i + 1) + count(nodes[i].w1) + 1u;
        };
        uint32_t nn = count(0);
        std::vector<Node> compact(nn);
        std::vector<uint32_t> acc(nodes.size());
        for (int64_t i = (int64_t)nn - 1, j = (int64_t)nodes.size(), skipped = 0; i >= 0; --i) {
            while (nodes[--j].w0 == 0 && nodes[j].w1 == 0) skipped++;
            Node &x = compact[i];
            x = nodes[j];
            acc[j] = (uint32_t)skipped;
            if (!(x.w0 & 1u)) x.w1 = (uint32_t)(i + x.w1 - j - (skipped - acc[x.w1]));
        }
        for (auto &x : compact) {
            BNode b;
            b.w0 = x.w0;
            b.w1 = x.w1;
            for (int i = 0; i < 3; ++i) { b.mn[i] = x.box.mn[i]; b.mx[i] = x.box.mx[i]; }
            s->nodes.push_back(b);
        }
    }
    *out = s.release();
    return NH_OK;
}

void no_scene_free(no_scene *s) { delete s; }

// Eigen's Vector4f::lpNorm<1>() = cwiseAbs().sum(): one SSE packet reduced as (x0 + x2) + (x1 + x3)
// (pinned against ext/eigen by oracle/eigen_probe.cpp)
static float l1_norm4(float x0, float x1, float x2, float x3) {
    return (std::fabs(x0) + std::fabs(x2)) + (std::fabs(x1) + std::fabs(x3));
}

// ---------------------------------------------------------------------------------------------------
// SimpleDenoiser (src/denoiser/simple.cpp) on an ImageBlock of (W + 2b) x (H + 2b) RGBW pixels, serial:
// the reference's loops run with one TBB thread (with several, its in-place rows race).
// ---------------------------------------------------------------------------------------------------
namespace {
constexpr float kNoriEpsilon = 1e-4f;

// Color4f::divideByFilterWeight().getLuminance() (color.h:113-118, common.cpp:265-268)
float block_luminance(const float *px) {
    float r = 0.f, g = 0.f, b = 0.f;
    if (std::fabs(px[3]) > kNoriEpsilon) { r = px[0] / px[3]; g = px[1] / px[3]; b = px[2] / px[3]; }
    return r * 0.212671f + g * 0.715160f + b * 0.072169f;
}

// computeVarianceFromImage (src/utils/common.cpp:339-398): 3x3 luminance variance, then normalised to
// [1, 1.254] (or all zero). std::pow(float, 2) is the double-precision pow of C++11's promotion rules, so
// each term and the running sum are evaluated in double and stored back to float.
std::vector<float> denoise_variance(const float *blk, int W, int H, int bs) {
    const int cols = W + 2 * bs;
    auto at = [&](int i, int j) { return blk + 4 * ((size_t)(i + bs) * cols + (j + bs)); };
    std::vector<float> var((size_t)W * H, 0.f);
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            float mean = 0.f, sum = 0.f;
            for (int k = 0; k < 3; ++k)
                for (int l = 0; l < 3; ++l) {
                    const int i_ = i - 1 + k, j_ = j - 1 + l;
                    if (i_ < 0 || i_ > H - 1 || j_ < 0 || j_ > W - 1) continue;
                    mean += std::fabs(block_luminance(at(i_, j_)));
                    sum += 1.f;
                }
            mean /= sum;
            float col = 0.f;
            for (int k = 0; k < 3; ++k)
                for (int l = 0; l < 3; ++l) {
                    const int i_ = i - 1 + k, j_ = j - 1 + l;
                    if (i_ < 0 || i_ > H - 1 || j_ < 0 || j_ > W - 1) continue;
                    const double d = (double)(std::fabs(block_luminance(at(i_, j_))) - mean);
                    col = (float)((double)col + (double)(1.f / sum) * (d * d));
                }
            var[(size_t)i * W + j] = col;
        }
    float mx = var[0], mn = var[0];
    for (float v : var) { mx = std::max(mx, v); mn = std::min(mn, v); }
    if (mx - mn < kNoriEpsilon) {
        std::fill(var.begin(), var.end(), 0.f);
    } else {
        for (float &v : var) v = 1.f + (v - mn) / (mx - mn) * 0.254f;
    }
    return var;
}
}  // namespace

int no_denoise_simple(float *rgbw, int32_t width, int32_t height, int32_t border, const nh_denoiser *p) {
    if (!rgbw || !p || width <= 0 || height <= 0 || border < 0 || p->type != NH_DENOISER_SIMPLE) return NH_ERR_INVALID;
    const int W = width, H = height, bs = border, cols = W + 2 * bs, r = p->range;
    const float sigma_d = p->sigma_d, sigma_vr = p->sigma_vr;
    auto at = [&](int i, int j) { return rgbw + 4 * ((size_t)(i + bs) * cols + (j + bs)); };
    for (int pass = 0; pass < p->amount; ++pass) {
        const std::vector<float> var = denoise_variance(rgbw, W, H, bs);
        for (int i = 0; i < H; ++i)
            for (int j = 0; j < W; ++j) {
                float sum_weights = 0.f, result[4] = {0.f, 0.f, 0.f, 0.f};
                const int i_s = std::clamp(i - r, 0, H), i_e = std::clamp(i + r + 1, 0, H);
                const int j_s = std::clamp(j - r, 0, W), j_e = std::clamp(j + r + 1, 0, W);
                const float vp = var[(size_t)i * W + j];
                for (int i_ = i_s; i_ < i_e; ++i_)
                    for (int j_ = j_s; j_ < j_e; ++j_) {
                        // g_sigma (simple.cpp:136-139): float expf of -(squaredNorm) / 2 / sigma_d / sigma_d
                        const int dsq = (i - i_) * (i - i_) + (j - j_) * (j - j_);
                        const float g = std::exp((float)-dsq / 2.f / sigma_d / sigma_d);
                        // f_prime (:140-149): p's current value (not yet overwritten) against q's current one
                        const float *ip = at(i, j), *iq = at(i_, j_);
                        const float l1 = l1_norm4(ip[0] - iq[0], ip[1] - iq[1], ip[2] - iq[2], ip[3] - iq[3]);
                        const float x = (l1 * vp) / sigma_vr;
                        const float f = (float)std::exp(-0.5f * ((double)x * (double)x));
                        const float w = g * f;
                        for (int k = 0; k < 4; ++k) result[k] += iq[k] * w;
                        sum_weights += w;
                    }
                float *op = at(i, j);
                for (int k = 0; k < 4; ++k) op[k] = result[k] / sum_weights;
            }
    }
    return NH_OK;
}

// The oracle's restated Eigen arithmetic on the probe's cases (oracle/eigen_probe.cpp layout): the same
// helpers the path uses (dot, normalized, max_coeff, sqnorm, norm, cross, cwise chains; camera_ray's
// 3x3 direction product and 4x4 point product)
int no_normal_ops(int32_t n, const float *in, float *out) {
    for (int32_t i = 0; i < n; ++i) {
        const float *p = in + 13 * (size_t)i;
        const V3 sv = mk(p[0], p[1], p[2]), tv = mk(p[3], p[4], p[5]), nv = mk(p[6], p[7], p[8]), v = mk(p[9], p[10], p[11]);
        float *o = out + 15 * (size_t)i;
        const V3 m = tbn_normal(sv, tv, nv, v);
        Frame f;
        f.s = sv;
        f.t = tv;
        f.n = nv;
        const Frame r = sphere_reframe(f, v);
        const V3 bl = normal_blend(v, p[12]);
        const float vals[15] = {m.x, m.y, m.z, r.n.x, r.n.y, r.n.z, r.s.x, r.s.y, r.s.z, r.t.x, r.t.y, r.t.z, bl.x, bl.y, bl.z};
        std::memcpy(o, vals, sizeof(vals));
    }
    return NH_OK;
}

int no_eigen_ops(int32_t n, const float *in, float *out) {
    for (int32_t i = 0; i < n; ++i) {
        const float *p = in + 36 * (size_t)i;
        const V3 a = mk(p[0], p[1], p[2]), b = mk(p[3], p[4], p[5]), c = mk(p[6], p[7], p[8]);
        const float s = p[9], *m3 = p + 10, *m4 = p + 20;
        float *o = out + 28 * (size_t)i;
        o[0] = dot(a, b);
        const V3 an = normalized(a);
        o[1] = an.x; o[2] = an.y; o[3] = an.z;
        o[4] = max_coeff(a);
        for (int r = 0; r < 3; ++r) o[5 + r] = m3[3 * r] * b.x + (m3[3 * r + 1] * b.y + m3[3 * r + 2] * b.z);
        const float v4[4] = {b.x, b.y, b.z, 1.0f};
        for (int r = 0; r < 4; ++r) {
            float acc = m4[4 * r + 0] * v4[0];
            acc = acc + m4[4 * r + 1] * v4[1];
            acc = acc + m4[4 * r + 2] * v4[2];
            acc = acc + m4[4 * r + 3] * v4[3];
            o[8 + r] = acc;
        }
        o[12] = sqnorm(a);
        o[13] = norm(a);
        const V3 ch = cmul(a * s, b);
        o[14] = ch.x; o[15] = ch.y; o[16] = ch.z;
        const V3 ch2 = cmul(cmul(a, b), c);
        o[17] = ch2.x; o[18] = ch2.y; o[19] = ch2.z;
        const V3 x = cross(a, b);
        o[20] = x.x; o[21] = x.y; o[22] = x.z;
        o[23] = norm(a - b);
        o[24] = l1_norm4(a.x - b.x, a.y - b.y, a.z - b.z, c.x - s);
        o[25] = a.x / s; o[26] = a.y / s; o[27] = a.z / s;
    }
    return NH_OK;
}

int no_bvh_info(const no_scene *s, uint32_t *n_nodes, uint32_t *n_indices) {
    *n_nodes = (uint32_t)s->nodes.size();
    *n_indices = (uint32_t)s->indices.size();
    return NH_OK;
}

int no_bvh_export(const no_scene *s, nh_bvh_node *nodes, uint32_t *indices) {
    for (size_t i = 0; i < s->nodes.size(); ++i) {
        nodes[i].word0 = s->nodes[i].w0;
        nodes[i].word1 = s->nodes[i].w1;
        for (int k = 0; k < 3; ++k) { nodes[i].bbox_min[k] = s->nodes[i].mn[k]; nodes[i].bbox_max[k] = s->nodes[i].mx[k]; }
    }
    std::memcpy(indices, s->indices.data(), s->indices.size() * sizeof(uint32_t));
    return NH_OK;
}

int no_trace_rays(const no_scene *s, const nh_ray_soa *r, int32_t n, int32_t any_hit, nh_hit_soa *out) {
    for (int32_t i = 0; i < n; ++i) {
        Ray ray = make_ray(mk(r->ox[i], r->oy[i], r->oz[i]), mk(r->dx[i], r->dy[i], r->dz[i]), r->mint[i], r->maxt[i]);
        Its its;
        uint32_t prim = 0;
        float bary[2] = {0.f, 0.f};
        bool hit = bvh_intersect(*s, ray, its, any_hit != 0, &prim, bary);
        out->hit[i] = hit ? 1 : 0;
        if (!any_hit) {  // u, v: Moller-Trumbore barycentrics (spheres: 0)
            out->t[i] = hit ? its.t : INFINITY;
            out->u[i] = hit ? bary[0] : 0.f;
            out->v[i] = hit ? bary[1] : 0.f;
            if (out->prim) out->prim[i] = hit ? prim : 0xffffffffu;
            if (out->shape) out->shape[i] = hit ? (uint32_t)its.shape : 0xffffffffu;
        }
    }
    return NH_OK;
}

void no_pcg32_seed(uint64_t *state, uint64_t *inc, uint64_t initstate, uint64_t initseq) {
    Pcg32 r;
    r.seed(initstate, initseq);
    *state = r.state;
    *inc = r.inc;
}
uint32_t no_pcg32_next(uint64_t *state, uint64_t *inc) {
    Pcg32 r;
    r.state = *state;
    r.inc = *inc;
    uint32_t v = r.next_uint();
    *state = r.state;
    return v;
}
void no_path_seed(uint64_t seed, uint64_t pixel_index, uint64_t sample_index, uint64_t *state, uint64_t *inc) {
    Pcg32 r;
    path_seed(r, seed, pixel_index, sample_index);
    *state = r.state;
    *inc = r.inc;
}

int no_path_radiance(const no_scene *s, uint64_t seed, int32_t px, int32_t py, int32_t sample, float *rgb3,
                     float *jitter2) {
    Sampler smp;
    path_seed(smp.rng, seed, (uint64_t)py * (uint64_t)s->cam.width + (uint64_t)px, (uint64_t)sample);
    float jx, jy, ax, ay;
    smp.next2d(jx, jy);
    smp.next2d(ax, ay);  // apertureSample (render.cpp:443), unused without DOF
    float spx = (float)px + jx, spy = (float)py + jy;
    float lens[2] = {0.f, 0.f};
    if (has_dof(s->cam)) {
        const int W = s->cam.width, H = s->cam.height;
        const uint64_t pos = serial_ray_index(W, H, 32)[(size_t)py * W + px];
        lens_jump(s->cam, (uint64_t)(uint32_t)sample * (uint64_t)W * (uint64_t)H + pos, lens);
    }
    Ray ray = camera_ray(s->cam, spx, spy, lens);
    V3 v = li(*s, smp, ray);
    rgb3[0] = v.x; rgb3[1] = v.y; rgb3[2] = v.z;
    if (jitter2) { jitter2[0] = jx; jitter2[1] = jy; }
    return NH_OK;
}

int no_render(const no_scene *s, int32_t mode, uint64_t seed, int32_t s0, int32_t s1, const int32_t *blocks,
              int32_t n_blocks, int32_t n_threads, float *rgbw, uint64_t *n_invalid) {
    if (!s || !rgbw || s1 < s0) return NH_ERR_INVALID;
    // NO_RENDER_LENS_SERIAL: the lens samples come from one sequential stream in the serial loop itself, literally
    // as the reference's single-thread render draws them (needs the whole image, one thread, round 0 onwards)
    const bool lens_serial = (mode & NO_RENDER_LENS_SERIAL) != 0;
    mode &= ~NO_RENDER_LENS_SERIAL;
    if (lens_serial && (blocks || n_threads != 1 || s0 != 0)) return NH_ERR_INVALID;
    if (mode == NO_SAMPLER_NORI_BLOCK && s0 != 0) return NH_ERR_INVALID;
    const int W = s->cam.width, H = s->cam.height, B = 32, border = s->filter.border;
    const bool dof = has_dof(s->cam);
    const std::vector<uint32_t> ray_pos = dof ? serial_ray_index(W, H, B) : std::vector<uint32_t>();
    Pcg32 lens_stream;  // the camera's static sampler (perspective.cpp:118-119), NO_RENDER_LENS_SERIAL only
    const int nbx = (W + B - 1) / B;
    auto order = spiral_blocks(W, H, B);
    std::vector<char> keep(order.size() ? (size_t)nbx * ((H + B - 1) / B) : 0, blocks ? 0 : 1);
    if (blocks)
        for (int i = 0; i < n_blocks; ++i) keep[blocks[i]] = 1;
    std::vector<std::pair<int, int>> work;
    for (auto &b : order)
        if (keep[(size_t)b.second * nbx + b.first]) work.push_back(b);
    std::vector<Block> bufs(work.size());
    std::vector<Pcg32> block_rng(work.size());
    for (size_t k = 0; k < work.size(); ++k) {
        Block &b = bufs[k];
        b.ox = work[k].first * B;
        b.oy = work[k].second * B;
        b.sx = std::min(B, W - b.ox);
        b.sy = std::min(B, H - b.oy);
        b.id = work[k].second * nbx + work[k].first;
        b.cols = b.rows = B + 2 * border;
        b.px.assign(4 * (size_t)b.cols * b.rows, 0.f);
        block_rng[k].seed((uint64_t)b.ox, (uint64_t)b.oy);  // Independent::prepare (independent.cpp:55-60)
    }
    std::atomic<uint64_t> invalid{0};
    const int64_t mcols = W + 2 * border;
    for (int32_t smp_i = s0; smp_i < s1; ++smp_i) {
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (;;) {
                size_t k = next.fetch_add(1);
                if (k >= work.size()) break;
                Block &b = bufs[k];
                std::fill(b.px.begin(), b.px.end(), 0.f);
                Sampler blk;
                blk.rng = block_rng[k];
                for (int x = 0; x < b.sx; ++x)  // getSampleIndices order (independent.cpp:93-99)
                    for (int y = 0; y < b.sy; ++y) {
                        Sampler per_path;
                        Sampler &smp = (mode == NO_SAMPLER_NORI_BLOCK) ? blk : per_path;
                        int px = x + b.ox, py = y + b.oy;
                        if (mode != NO_SAMPLER_NORI_BLOCK)
                            path_seed(per_path.rng, seed, (uint64_t)py * (uint64_t)W + (uint64_t)px, (uint64_t)smp_i);
                        float jx, jy, ax, ay;
                        smp.next2d(jx, jy);
                        smp.next2d(ax, ay);
                        float spx = (float)px + jx, spy = (float)py + jy;
                        float lens[2] = {0.f, 0.f};
                        if (dof && lens_serial) {
                            const float a = lens_stream.next_float(), b = lens_stream.next_float();  // next2D()
                            lens[0] = s->cam.lens_draw_order == NH_LENS_DRAWS_RTL ? b : a;
                            lens[1] = s->cam.lens_draw_order == NH_LENS_DRAWS_RTL ? a : b;
                        } else if (dof) {
                            lens_jump(s->cam, (uint64_t)(uint32_t)smp_i * (uint64_t)W * (uint64_t)H +
                                          ray_pos[(size_t)py * W + px], lens);
                        }
                        Ray ray = camera_ray(s->cam, spx, spy, lens);
                        V3 v = li(*s, smp, ray);
                        v = v * 1.0f;  // value = Color3f(1) * Li
                        if (!block_put(b, s->filter, spx, spy, v)) invalid++;
                    }
                block_rng[k] = blk.rng;
            }
        };
        int nt = std::max(1, n_threads);
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(worker);
        worker();
        for (auto &t : th) t.join();
        // master.put(block) in spiral order (block.cpp:125-134): offset (ox, oy) in master array coords
        for (auto &b : bufs) {
            int rows = b.sy + 2 * border, cols = b.sx + 2 * border;
            for (int y = 0; y < rows; ++y)
                for (int x = 0; x < cols; ++x) {
                    float *m = &rgbw[4 * ((int64_t)(b.oy + y) * mcols + (b.ox + x))];
                    const float *p = &b.px[4 * ((size_t)y * b.cols + x)];
                    m[0] += p[0]; m[1] += p[1]; m[2] += p[2]; m[3] += p[3];
                }
        }
    }
    if (n_invalid) *n_invalid = invalid.load();
    return NH_OK;
}

int no_ttest_scene(const no_scene *s, uint64_t *state, uint64_t *inc, int32_t n, double *mean, double *variance) {
    Sampler smp;
    smp.rng.state = *state;
    smp.rng.inc = *inc;
    double m = 0, var = 0;
    for (int32_t k = 0; k < n; ++k) {
        float a, b;
        smp.next2d(a, b);
        float spx = a * (float)s->cam.width, spy = b * (float)s->cam.height;
        float ax, ay;
        smp.next2d(ax, ay);
        float lens[2] = {0.f, 0.f};
        if (has_dof(s->cam)) lens_jump(s->cam, (uint64_t)k, lens);  // the k-th sampleRay of this serial loop
        Ray ray = camera_ray(s->cam, spx, spy, lens);
        V3 v = li(*s, smp, ray);
        double r = (double)luminance(v);
        double delta = r - m;
        m += delta / (double)(k + 1);
        var += delta * (r - m);
    }
    var /= n - 1;
    *mean = m;
    *variance = var;
    *state = smp.rng.state;
    *inc = smp.rng.inc;
    return NH_OK;
}

int no_ttest_bsdf(const nh_bsdf *b, float angle_deg, uint64_t *state, uint64_t *inc, int32_t n, double *mean,
                  double *variance) {
    Pcg32 rng;
    rng.state = *state;
    rng.inc = *inc;
    // sphericalDirection(degToRad(angle), 0) (common.cpp:270-281): sincosf; degToRad promotes to double
    // (common.h:218: value * (M_PI / 180.0f))
    float theta = (float)((double)angle_deg * (3.14159265358979323846 / (double)180.0f));
    float st = f_sin(theta), ct = f_cos(theta), sp = f_sin(0.f), cp = f_cos(0.f);
    V3 wi = mk(st * cp, st * sp, ct);
    double m = 0, var = 0;
    for (int32_t k = 0; k < n; ++k) {
        float a = rng.next_float();
        float c = rng.next_float();
        BRec r;
        r.wi = wi;
        double res = (double)luminance(bsdf_sample(*b, r, a, c));
        double delta = res - m;
        m += delta / (double)(k + 1);
        var += delta * (res - m);
    }
    var /= n - 1;
    *mean = m;
    *variance = var;
    *state = rng.state;
    *inc = rng.inc;
    return NH_OK;
}

int no_bsdf_sample(const nh_bsdf *b, const float *wi, const float *sample, float *wo, float *weight3, float *pdf,
                   int32_t *measure) {
    BRec r;
    r.wi = mk(wi[0], wi[1], wi[2]);
    V3 w = bsdf_sample(*b, r, sample[0], sample[1]);
    wo[0] = r.wo.x; wo[1] = r.wo.y; wo[2] = r.wo.z;
    weight3[0] = w.x; weight3[1] = w.y; weight3[2] = w.z;
    *pdf = bsdf_pdf(*b, r);
    *measure = (int32_t)r.measure;
    return NH_OK;
}

// ChiSquareTest::execute sampling loop (src/utils/chi2test.cpp:150-170): histogram of
// sample() directions over cos(theta) x phi cells; rng state in/out.
int no_chi2_histogram(const nh_bsdf *b, const float *wi, uint64_t *state, uint64_t *inc, int32_t n, int32_t res_theta,
                      int32_t res_phi, double *obs) {
    Pcg32 rng;
    rng.state = *state;
    rng.inc = *inc;
    BRec r;
    r.wi = mk(wi[0], wi[1], wi[2]);
    for (int32_t i = 0; i < n; ++i) {
        float a = rng.next_float();
        float c = rng.next_float();
        V3 res = bsdf_sample(*b, r, a, c);
        if (res.x == 0 && res.y == 0 && res.z == 0) continue;
        int ct = std::min(std::max(0, (int)std::floor((r.wo.z * 0.5f + 0.5f) * res_theta)), res_theta - 1);
        float scaled_phi = f_atan2(r.wo.y, r.wo.x) * 0.15915494309189533577f;
        if (scaled_phi < 0) scaled_phi += 1;
        int pb = std::min(std::max(0, (int)std::floor(scaled_phi * res_phi)), res_phi - 1);
        obs[ct * res_phi + pb] += 1;
    }
    *state = rng.state;
    *inc = rng.inc;
    return NH_OK;
}

int no_texture_eval(const no_scene *s, uint32_t texture, int32_t n, const float *u, const float *v, float *rgb) {
    if (!s || texture == 0 || texture > s->textures.size() || n < 0) return NH_ERR_INVALID;
    for (int32_t i = 0; i < n; ++i) {
        const V3 c = texture_eval(*s, s->textures[texture - 1], u[i], v[i]);
        rgb[3 * i] = c.x;
        rgb[3 * i + 1] = c.y;
        rgb[3 * i + 2] = c.z;
    }
    return NH_OK;
}

int no_bsdf_pdf_batch(const nh_bsdf *b, const float *wi, int32_t n, const float *wo, float *out) {
    for (int32_t i = 0; i < n; ++i) {
        BRec r;
        r.wi = mk(wi[0], wi[1], wi[2]);
        r.wo = mk(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
        r.measure = ESolidAngle;
        out[i] = bsdf_pdf(*b, r);
    }
    return NH_OK;
}

float no_bsdf_pdf(const nh_bsdf *b, const float *wi, const float *wo) {
    BRec r;
    r.wi = mk(wi[0], wi[1], wi[2]);
    r.wo = mk(wo[0], wo[1], wo[2]);
    r.measure = ESolidAngle;
    return bsdf_pdf(*b, r);
}

}  // extern "C"
