// Host-side transform arithmetic of the reference's scene setup, restated in plain C++ with the exact
// float operations its vendored Eigen 3.3.8 performs on x86-64 (SSE2, no FMA contraction), so that
// camera matrices and baked mesh vertices are bit-identical to the reference's:
//   - the parser's transform composition (src/utils/parser.cpp:308-360), each operation pre-multiplied
//     onto an Eigen::Affine3f:
//       Translation * T    -> T.translation() += v                       (Eigen Translation.h:125-130)
//       Diagonal * T       -> rows of T's linear part and translation scaled (Eigen Transform.h, diagonal
//                             product)
//       AngleAxis * T      -> toRotationMatrix() * T.topRows<3>()        (RotationBase.h:89-90,
//                             Transform.h:1460-1474, AngleAxis.h:218-245)
//       Affine3f(M) * T    -> linear = L_M * L_T, translation = L_M * t_T + t_M (Transform.h:1481-1495)
//   - nori::Transform(Matrix4f) stores Matrix4f::inverse(), Eigen's SSE 4x4 float inverse
//     (ext/eigen/Eigen/src/LU/arch/Inverse_SSE.h:35-163, Intel's 2x2-block "divide and conquer"
//     formula with one scalar reciprocal of the determinant), restated lane by lane below;
//   - Transform * Point3f / Vector3f / Normal3f (include/nori/transform.h:73-86);
//   - PerspectiveCamera::update's sampleToCamera (src/cameras/perspective.cpp:68-95).
// Eigen's evaluation orders (pinned against the real Eigen by tests/test_transforms.py through
// oracle/_ref/eigen_xform_probe): small coefficient-based products of inner size 3 sum
// p0 + (p1 + p2) (the unrolled redux halves 3 as 1 + 2), 4x4 * 4-vector products (SSE packets)
// sum left to right; float sin / cos / tan are the C library's float functions, as Eigen calls them.
#pragma once

#include <cmath>

namespace nh {
namespace xf {

// row-major 4x4 float matrix
struct Mat4 {
    float m[4][4];
    static Mat4 identity() {
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.m[i][j] = (i == j) ? 1.0f : 0.0f;
        return r;
    }
};

struct Vec3 {
    float x, y, z;
};

// include/nori/common.h:218 -- degToRad promotes to double: value * (M_PI / 180.0f), rounded once
inline float deg_to_rad(float value) { return (float)((double)value * (3.14159265358979323846 / (double)180.0f)); }

// Eigen redux of a length-3 product: p0 + (p1 + p2)
inline float dot3(float a0, float a1, float a2, float b0, float b1, float b2) { return a0 * b0 + (a1 * b1 + a2 * b2); }

inline Vec3 normalized(Vec3 a) {  // MatrixBase::normalized: divide by sqrt(squaredNorm) when > 0
    const float n = dot3(a.x, a.y, a.z, a.x, a.y, a.z);
    if (n > 0.0f) {
        const float s = std::sqrt(n);
        return {a.x / s, a.y / s, a.z / s};
    }
    return a;
}
inline Vec3 cross(Vec3 a, Vec3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

// ---- parser operations on an Affine3f (only the top three rows matter; row 3 stays 0 0 0 1) ----

inline void pre_translate(Mat4 &t, Vec3 v) {  // Translation * T
    t.m[0][3] = t.m[0][3] + v.x;
    t.m[1][3] = t.m[1][3] + v.y;
    t.m[2][3] = t.m[2][3] + v.z;
}

inline void pre_scale(Mat4 &t, Vec3 v) {  // DiagonalMatrix * T: linear and translation rows scaled
    const float d[3] = {v.x, v.y, v.z};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) t.m[i][j] = d[i] * t.m[i][j];
}

// AngleAxis<float>(angle, axis).toRotationMatrix(); the axis is used as given (not normalised)
inline void angle_axis_matrix(float angle, Vec3 a, float r[3][3]) {
    const float s = std::sin(angle), c = std::cos(angle);
    const Vec3 sa = {s * a.x, s * a.y, s * a.z};
    const Vec3 c1 = {(1.0f - c) * a.x, (1.0f - c) * a.y, (1.0f - c) * a.z};
    float tmp = c1.x * a.y;
    r[0][1] = tmp - sa.z;
    r[1][0] = tmp + sa.z;
    tmp = c1.x * a.z;
    r[0][2] = tmp + sa.y;
    r[2][0] = tmp - sa.y;
    tmp = c1.y * a.z;
    r[1][2] = tmp - sa.x;
    r[2][1] = tmp + sa.x;
    r[0][0] = c1.x * a.x + c;
    r[1][1] = c1.y * a.y + c;
    r[2][2] = c1.z * a.z + c;
}

inline void pre_rotate(Mat4 &t, float angle, Vec3 axis) {  // R * T.topRows<3>()
    float r[3][3];
    angle_axis_matrix(angle, axis, r);
    Mat4 o = t;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) o.m[i][j] = dot3(r[i][0], r[i][1], r[i][2], t.m[0][j], t.m[1][j], t.m[2][j]);
    t = o;
}

// Affine3f(M) * T (only M's top three rows are read)
inline void pre_affine(Mat4 &t, const Mat4 &a) {
    Mat4 o = Mat4::identity();
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) o.m[i][j] = dot3(a.m[i][0], a.m[i][1], a.m[i][2], t.m[0][j], t.m[1][j], t.m[2][j]);
        o.m[i][3] = dot3(a.m[i][0], a.m[i][1], a.m[i][2], t.m[0][3], t.m[1][3], t.m[2][3]) + a.m[i][3];
    }
    t = o;
}

// PNGTexture's spherical-lookup rotation (PNGTexture.cpp:28, :133-139):
//   eulerAngles = degrees * M_PI / 180.f;
//   rot = Quaternionf(Identity * AngleAxisf(e.x, UnitZ) * AngleAxisf(e.y, UnitX)) * AngleAxisf(e.z, UnitZ).toRotationMatrix()
// in Eigen 3.3.8's float arithmetic: AngleAxis -> Quaternion (Quaternion.h:523-531), the SSE quaternion product
// (arch/Geometry_SSE.h quat_product), Quaternion::toRotationMatrix (Quaternion.h:554-586), AngleAxis::
// toRotationMatrix (AngleAxis.h:218-242) and the 3x3 product in the order Eigen's lazy product gives. Pinned by
// oracle/eigen_xform_probe.cpp ("prot"). Row-major out[9].
struct Quat {
    float x, y, z, w;
};
inline Quat quat_from_angle_axis(float angle, Vec3 axis) {
    const float ha = 0.5f * angle;
    const float s = std::sin(ha);
    return {s * axis.x, s * axis.y, s * axis.z, std::cos(ha)};
}
inline Quat quat_mul(Quat a, Quat b) {  // _mm_add_ps(_mm_sub_ps(a * b.wwww, a.zxyx * b.yzxx), mask ^ (s1 + s2))
    const float s1[4] = {a.y * b.z, a.z * b.x, a.x * b.y, a.z * b.z};
    const float s2[4] = {a.w * b.x, a.w * b.y, a.w * b.z, a.y * b.y};
    const float t1[4] = {a.x * b.w, a.y * b.w, a.z * b.w, a.w * b.w};
    const float t2[4] = {a.z * b.y, a.x * b.z, a.y * b.x, a.x * b.x};
    return {(t1[0] - t2[0]) + (s1[0] + s2[0]), (t1[1] - t2[1]) + (s1[1] + s2[1]), (t1[2] - t2[2]) + (s1[2] + s2[2]),
            (t1[3] - t2[3]) + -(s1[3] + s2[3])};
}
inline void quat_matrix(Quat q, float r[3][3]) {
    const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z;
    const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    r[0][0] = 1.f - (tyy + tzz);
    r[0][1] = txy - twz;
    r[0][2] = txz + twy;
    r[1][0] = txy + twz;
    r[1][1] = 1.f - (txx + tzz);
    r[1][2] = tyz - twx;
    r[2][0] = txz - twy;
    r[2][1] = tyz + twx;
    r[2][2] = 1.f - (txx + tyy);
}
inline void png_rotation(Vec3 deg, float out[9]) {
    const float pi = 3.14159265358979323846f;  // Nori's float M_PI (common.h:61)
    const Vec3 e = {deg.x * pi / 180.f, deg.y * pi / 180.f, deg.z * pi / 180.f};
    const Vec3 ux = {1.f, 0.f, 0.f}, uz = {0.f, 0.f, 1.f};
    const Quat q = quat_mul(quat_mul(Quat{0.f, 0.f, 0.f, 1.f}, quat_from_angle_axis(e.x, uz)), quat_from_angle_axis(e.y, ux));
    float a[3][3], b[3][3];
    quat_matrix(q, a);
    angle_axis_matrix(e.z, uz, b);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = dot3(a[i][0], a[i][1], a[i][2], b[0][j], b[1][j], b[2][j]);
}

// parser.cpp:343-359: columns left, newUp, dir, origin
inline Mat4 lookat_matrix(Vec3 origin, Vec3 target, Vec3 up) {
    const Vec3 dir = normalized({target.x - origin.x, target.y - origin.y, target.z - origin.z});
    const Vec3 left = normalized(cross(normalized(up), dir));
    const Vec3 new_up = normalized(cross(dir, left));
    Mat4 r = Mat4::identity();
    const Vec3 cols[4] = {left, new_up, dir, origin};
    for (int j = 0; j < 4; ++j) {
        r.m[0][j] = cols[j].x;
        r.m[1][j] = cols[j].y;
        r.m[2][j] = cols[j].z;
    }
    return r;
}

// ---- Matrix4f::inverse(), SSE float path: Eigen's packets are the columns of the column-major matrix ----

struct F4 {
    float v[4];
};
inline F4 f4(float a, float b, float c, float d) { return {{a, b, c, d}}; }
inline F4 mul(F4 a, F4 b) { return f4(a.v[0] * b.v[0], a.v[1] * b.v[1], a.v[2] * b.v[2], a.v[3] * b.v[3]); }
inline F4 add(F4 a, F4 b) { return f4(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3]); }
inline F4 sub(F4 a, F4 b) { return f4(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2], a.v[3] - b.v[3]); }
inline F4 sub_ss(F4 a, F4 b) { a.v[0] = a.v[0] - b.v[0]; return a; }
inline F4 add_ss(F4 a, F4 b) { a.v[0] = a.v[0] + b.v[0]; return a; }
inline F4 mul_ss(F4 a, F4 b) { a.v[0] = a.v[0] * b.v[0]; return a; }
// _mm_shuffle_ps(a, b, imm): two lanes of a, then two of b
inline F4 shuf(F4 a, F4 b, int imm) {
    return f4(a.v[imm & 3], a.v[(imm >> 2) & 3], b.v[(imm >> 4) & 3], b.v[(imm >> 6) & 3]);
}
inline F4 movelh(F4 a, F4 b) { return f4(a.v[0], a.v[1], b.v[0], b.v[1]); }
inline F4 movehl(F4 a, F4 b) { return f4(b.v[2], b.v[3], a.v[2], a.v[3]); }
inline F4 splat0(F4 a) { return f4(a.v[0], a.v[0], a.v[0], a.v[0]); }

inline Mat4 inverse(const Mat4 &in) {
    F4 col[4];
    for (int j = 0; j < 4; ++j) col[j] = f4(in.m[0][j], in.m[1][j], in.m[2][j], in.m[3][j]);
    // the four 2x2 blocks, each packed column-major
    const F4 A = movelh(col[0], col[1]), B = movehl(col[1], col[0]);
    const F4 C = movelh(col[2], col[3]), D = movehl(col[3], col[2]);
    // adj(A) * B and adj(D) * C
    F4 AB = mul(shuf(A, A, 0x0F), B);
    AB = sub(AB, mul(shuf(A, A, 0xA5), shuf(B, B, 0x4E)));
    F4 DC = mul(shuf(D, D, 0x0F), C);
    DC = sub(DC, mul(shuf(D, D, 0xA5), shuf(C, C, 0x4E)));
    // 2x2 determinants in lane 0
    F4 dA = mul(shuf(A, A, 0x5F), A);
    dA = sub_ss(dA, movehl(dA, dA));
    F4 dB = mul(shuf(B, B, 0x5F), B);
    dB = sub_ss(dB, movehl(dB, dB));
    F4 dC = mul(shuf(C, C, 0x5F), C);
    dC = sub_ss(dC, movehl(dC, dC));
    F4 dD = mul(shuf(D, D, 0x5F), D);
    dD = sub_ss(dD, movehl(dD, dD));
    F4 d = mul(shuf(DC, DC, 0xD8), AB);
    F4 iD = mul(shuf(C, C, 0xA0), movelh(AB, AB));
    iD = add(iD, mul(shuf(C, C, 0xF5), movehl(AB, AB)));
    F4 iA = mul(shuf(B, B, 0xA0), movelh(DC, DC));
    iA = add(iA, mul(shuf(B, B, 0xF5), movehl(DC, DC)));
    d = add(d, movehl(d, d));
    d = add_ss(d, shuf(d, d, 1));
    const F4 d1 = mul_ss(dA, dD), d2 = mul_ss(dB, dC);
    iD = sub(mul(D, splat0(dA)), iD);
    iA = sub(mul(A, splat0(dD)), iA);
    const F4 det = sub_ss(add_ss(d1, d2), d);
    const float rd0 = 1.0f / det.v[0];  // _mm_div_ss(_mm_set_ss(1), det)
    F4 iB = mul(D, shuf(AB, AB, 0x33));
    iB = sub(iB, mul(shuf(D, D, 0xB1), shuf(AB, AB, 0x66)));
    F4 iC = mul(A, shuf(DC, DC, 0x33));
    iC = sub(iC, mul(shuf(A, A, 0xB1), shuf(DC, DC, 0x66)));
    const F4 rd = f4(rd0, -rd0, -rd0, rd0);  // sign mask + - - +
    iB = sub(mul(C, splat0(dB)), iB);
    iC = sub(mul(B, splat0(dC)), iC);
    iA = mul(rd, iA);
    iB = mul(rd, iB);
    iC = mul(rd, iC);
    iD = mul(rd, iD);
    const F4 out[4] = {shuf(iA, iB, 0x77), shuf(iA, iB, 0x22), shuf(iC, iD, 0x77), shuf(iC, iD, 0x22)};
    Mat4 r;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) r.m[i][j] = out[j].v[i];
    return r;
}

// ---- applying a nori::Transform ----

// Transform * Point3f: (M * (p, 1)) left to right, then xyz / w
inline Vec3 apply_point(const Mat4 &t, Vec3 p) {
    float r[4];
    for (int i = 0; i < 4; ++i) {
        float s = t.m[i][0] * p.x;
        s = s + t.m[i][1] * p.y;
        s = s + t.m[i][2] * p.z;
        s = s + t.m[i][3] * 1.0f;
        r[i] = s;
    }
    return {r[0] / r[3], r[1] / r[3], r[2] / r[3]};
}
// Transform * Vector3f: topLeftCorner<3,3>() * v
inline Vec3 apply_vector(const Mat4 &t, Vec3 v) {
    return {dot3(t.m[0][0], t.m[0][1], t.m[0][2], v.x, v.y, v.z), dot3(t.m[1][0], t.m[1][1], t.m[1][2], v.x, v.y, v.z),
            dot3(t.m[2][0], t.m[2][1], t.m[2][2], v.x, v.y, v.z)};
}
// Transform * Normal3f: inverse.topLeftCorner<3,3>().transpose() * n
inline Vec3 apply_normal(const Mat4 &inv, Vec3 n) {
    return {dot3(inv.m[0][0], inv.m[1][0], inv.m[2][0], n.x, n.y, n.z),
            dot3(inv.m[0][1], inv.m[1][1], inv.m[2][1], n.x, n.y, n.z),
            dot3(inv.m[0][2], inv.m[1][2], inv.m[2][2], n.x, n.y, n.z)};
}

// ---- PerspectiveCamera::update: the matrix whose inverse is sampleToCamera ----
// DiagonalMatrix(0.5, -0.5 aspect, 1) * Translation(1, -1/aspect, 0) is an Affine3f (Translation.h:112-121);
// Affine3f * Matrix4f keeps the perspective's last row and forms the top rows as affine() * P, a
// coefficient-based product of inner size 4 (Transform.h:1322-1345): (p0 + p1) + (p2 + p3).
inline Mat4 camera_projection(int width, int height, float fov, float near_clip, float far_clip) {
    const float aspect = (float)width / (float)height;
    const float recip = 1.0f / (far_clip - near_clip);
    const float cot = 1.0f / std::tan(deg_to_rad(fov / 2.0f));
    Mat4 p = Mat4::identity();
    p.m[0][0] = cot;
    p.m[1][1] = cot;
    p.m[2][2] = far_clip * recip;
    p.m[2][3] = -near_clip * far_clip * recip;
    p.m[3][2] = 1.0f;
    p.m[3][3] = 0.0f;
    const float dg[3] = {0.5f, -0.5f * aspect, 1.0f};
    const float tr[3] = {1.0f, -1.0f / aspect, 0.0f};
    float aff[3][4];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) aff[i][j] = (i == j) ? dg[i] : 0.0f;
        aff[i][3] = dg[i] * tr[i];
    }
    Mat4 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[i][j] = (aff[i][0] * p.m[0][j] + aff[i][1] * p.m[1][j]) + (aff[i][2] * p.m[2][j] + aff[i][3] * p.m[3][j]);
    for (int j = 0; j < 4; ++j) r.m[3][j] = p.m[3][j];
    return r;
}

}  // namespace xf
}  // namespace nh
