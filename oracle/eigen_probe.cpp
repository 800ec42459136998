// TEST INFRASTRUCTURE ONLY. Evaluation-order probe: compiled by oracle/build_ref.sh against the
// reference's own vendored Eigen 3.3.8 (/root/reference/ext/eigen, unmodified) with the reference's
// floating-point setup (x86-64 SSE2, no FMA contraction), it evaluates the Eigen expressions the
// reference's path uses and writes the float results, so tests/test_oracle_kat.py can check that the
// oracle's restated arithmetic (oracle/nori_oracle.cpp: dot, normalized, maxCoeff, cross, norms,
// 3x3 / 4x4 matrix-vector products, cwise Color3f chains, the SimpleDenoiser's Vector4f lpNorm<1> and
// Color4f::divideByFilterWeight's Color3f / w) is bit-identical to Eigen's.
//
// usage: eigen_probe IN OUT   IN: n x 36 floats per case (a3 b3 c3 s m3[9] pad m4[16]), OUT: n x 28 floats
#include <Eigen/Core>
#include <Eigen/Geometry>

#include <cstdio>
#include <vector>

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> in;
    float buf[36];
    while (std::fread(buf, sizeof(float), 36, f) == 36) in.insert(in.end(), buf, buf + 36);
    std::fclose(f);
    const size_t n = in.size() / 36;
    std::vector<float> out(n * 28, 0.f);
    for (size_t i = 0; i < n; ++i) {
        const float *p = &in[36 * i];
        const Eigen::Vector3f a(p[0], p[1], p[2]), b(p[3], p[4], p[5]), c(p[6], p[7], p[8]);
        const float s = p[9];
        Eigen::Matrix3f m3;  // row-major input
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) m3(r, k) = p[10 + 3 * r + k];
        Eigen::Matrix4f m4;
        for (int r = 0; r < 4; ++r)
            for (int k = 0; k < 4; ++k) m4(r, k) = p[20 + 4 * r + k];
        float *o = &out[28 * i];
        o[0] = a.dot(b);                          // Frame::toLocal / cosTheta, BSDF and light terms
        const Eigen::Vector3f an = a.normalized();  // ray directions, frames
        o[1] = an.x(); o[2] = an.y(); o[3] = an.z();
        o[4] = a.maxCoeff();                      // Russian roulette max(t)
        const Eigen::Vector3f mv = m3 * b;        // Transform of a vector (3x3 block)
        o[5] = mv.x(); o[6] = mv.y(); o[7] = mv.z();
        const Eigen::Vector4f v4(b.x(), b.y(), b.z(), 1.0f);
        const Eigen::Vector4f m4v = m4 * v4;      // Transform of a point (camera sampleToCamera, cameraToWorld)
        o[8] = m4v.x(); o[9] = m4v.y(); o[10] = m4v.z(); o[11] = m4v.w();
        o[12] = a.squaredNorm();
        o[13] = a.norm();
        const Eigen::Array3f ca = a.array(), cb = b.array(), cc = c.array();
        const Eigen::Array3f chain = (ca * s) * cb;  // Color3f li * cos * f
        o[14] = chain.x(); o[15] = chain.y(); o[16] = chain.z();
        const Eigen::Array3f chain2 = ca * cb * cc;  // t * bsdf * Le
        o[17] = chain2.x(); o[18] = chain2.y(); o[19] = chain2.z();
        const Eigen::Vector3f x = a.cross(b);
        o[20] = x.x(); o[21] = x.y(); o[22] = x.z();
        o[23] = (a - b).norm();                   // distances (emitter pdfs, shadow ray lengths)
        // SimpleDenoiser::f_prime colour distance (src/denoiser/simple.cpp:145-147)
        o[24] = Eigen::Vector4f(a.x() - b.x(), a.y() - b.y(), a.z() - b.z(), c.x() - s).lpNorm<1>();
        const Eigen::Array3f q = ca / s;          // Color4f::divideByFilterWeight (color.h:113-118)
        o[25] = q.x(); o[26] = q.y(); o[27] = q.z();
    }
    f = std::fopen(argv[2], "wb");
    if (!f) return 2;
    std::fwrite(out.data(), sizeof(float), out.size(), f);
    std::fclose(f);
    return 0;
}
