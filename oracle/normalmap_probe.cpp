// TEST INFRASTRUCTURE ONLY. Texture / normal-map probe: compiled by oracle/build_ref.sh against the reference's own
// vendored lodepng (/root/reference/ext/lodepng/src/lodepng.cpp) and Eigen 3.3.8 (ext/eigen), unmodified, with the
// reference's floating-point setup (x86-64 SSE2, no FMA contraction). It evaluates the expressions of the reference's
// texture and normal-map code with those libraries -- PNGTexture::loadFromFile's decode loops (PNGTexture.cpp:78-95),
// InverseGammaCorrect (:442-447), PNGTexture::eval's lookup and normal-map blend (:143-161), the mesh TBN product
// (mesh.cpp:173-183) and the sphere re-framing (sphere.cpp:115-121, Frame::toWorld frame.h:61-63) -- so
// tests/test_normalmap.py can pin the product loader (nh_texture_decode, png_decode.cpp) and the oracle
// (no_normal_ops) bit for bit. The PNGTexture / Mesh / Sphere classes themselves include nori/common.h
// (-> IlmBase's ImathPlatform.h, absent), so their expressions are restated here over the same Eigen types
// (Nori's Vector3f / Normal3f / Color3f are thin subclasses of Eigen::Matrix<float,3,1> / Eigen::Array<float,3,1>).
//
// usage:
//   normalmap_probe png  IN.png OUT srgb    lodepng::decode(RGBA8) + the decode loop: OUT = u32 w, u32 h, floats
//   normalmap_probe bytes IN OUT srgb       the decode loop over raw bytes: OUT = floats
//   normalmap_probe ops IN OUT              per case 13 floats (s3 t3 n3 v3 intensity) -> 15 floats:
//                                           normalize(TBN * v), sphere (n', t', b'), blend(v, intensity)
//   normalmap_probe order OUT               Point2f(nextFloat(), nextFloat()) with a Nori-shaped 2-vector
//                                           constructor: OUT = 2 floats of the first call from a default pcg32
#include <Eigen/Core>
#include <Eigen/Geometry>
#include <lodepng/lodepng.h>
#include <pcg32.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

// PNGTexture::InverseGammaCorrect, written as the reference writes it (PNGTexture.cpp:442-447)
float InverseGammaCorrect(float value) {
    if (value <= 0.04045f) return value * 1.f / 12.92f;
    return std::pow((value + 0.055f) * 1.f / 1.055f, 2.4f);
}

// PNGTexture::loadFromFile's loop over lodepng's bytes (PNGTexture.cpp:78-95)
void decode(const std::vector<unsigned char> &tmp, bool sRgb, std::vector<float> &data) {
    data.resize(tmp.size());
    if (sRgb) {
        for (unsigned int i = 0; i < data.size(); ++i) data[i] = InverseGammaCorrect(static_cast<float>(tmp[i]) / 255.f);
    } else {
        for (unsigned int i = 0; i < data.size(); ++i) {
            data[i] = static_cast<float>(tmp[i]) / 255 * 2 - 1;
            if ((i + 1) % 3 == 0) Eigen::Map<Eigen::Vector3f>(data.data() + i - 2).normalize();
        }
    }
}

bool write_all(const char *path, const void *p, size_t n) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, n, f) == n;
    return std::fclose(f) == 0 && ok;
}

// Nori's TPoint<float, 2> constructor shape (vector.h: TPoint(Scalar x, Scalar y)), out of line so the argument
// evaluation order is the compiler's choice at the call site, as in Independent::next2D (independent.cpp:74-78)
struct Point2 {
    float x, y;
    Point2(float x_, float y_) : x(x_), y(y_) {}
};

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const std::string mode = argv[1];
    if (mode == "png" || mode == "bytes") {
        if (argc != 5) return 2;
        const bool srgb = std::atoi(argv[4]) != 0;
        std::vector<unsigned char> tmp;
        unsigned w = 0, h = 0;
        if (mode == "png") {
            if (lodepng::decode(tmp, w, h, argv[2])) return 3;
        } else {
            FILE *f = std::fopen(argv[2], "rb");
            if (!f) return 2;
            int c;
            while ((c = std::fgetc(f)) != EOF) tmp.push_back((unsigned char)c);
            std::fclose(f);
        }
        std::vector<float> data;
        decode(tmp, srgb, data);
        std::vector<unsigned char> out;
        if (mode == "png") {
            const uint32_t wh[2] = {w, h};
            out.insert(out.end(), (const unsigned char *)wh, (const unsigned char *)wh + 8);
        }
        out.insert(out.end(), (const unsigned char *)data.data(), (const unsigned char *)(data.data() + data.size()));
        return write_all(argv[3], out.data(), out.size()) ? 0 : 2;
    }
    if (mode == "ops") {
        if (argc != 4) return 2;
        FILE *f = std::fopen(argv[2], "rb");
        if (!f) return 2;
        std::vector<float> in;
        float buf[13];
        while (std::fread(buf, sizeof(float), 13, f) == 13) in.insert(in.end(), buf, buf + 13);
        std::fclose(f);
        const size_t n = in.size() / 13;
        std::vector<float> out(n * 15);
        for (size_t i = 0; i < n; ++i) {
            const float *p = &in[13 * i];
            const Eigen::Vector3f s(p[0], p[1], p[2]), t(p[3], p[4], p[5]), nn(p[6], p[7], p[8]);
            const Eigen::Vector3f v(p[9], p[10], p[11]);
            const float intensity = p[12];
            float *o = &out[15 * i];
            // mesh.cpp:176-182: TBN << aTangent, aBitangent, normal; normal = (TBN * eval(uv)).normalized()
            Eigen::Matrix3f TBN;
            TBN << s, t, nn;
            Eigen::Vector3f normal = TBN * v;
            normal = normal.normalized();
            o[0] = normal.x(); o[1] = normal.y(); o[2] = normal.z();
            // sphere.cpp:117-120 with its.shFrame = Frame(s, t, n): Frame::toWorld = s * v.x() + t * v.y() + n * v.z()
            const Eigen::Vector3f sn = (s * v.x() + t * v.y() + nn * v.z()).normalized();
            const Eigen::Vector3f st = (Eigen::Vector3f(0, 0, 1).cross(sn)).normalized();
            const Eigen::Vector3f sb = sn.cross(st);
            o[3] = sn.x(); o[4] = sn.y(); o[5] = sn.z();
            o[6] = st.x(); o[7] = st.y(); o[8] = st.z();
            o[9] = sb.x(); o[10] = sb.y(); o[11] = sb.z();
            // PNGTexture::eval's normal-map branch (PNGTexture.cpp:155-161) on a texel v (Color3f = Array3f)
            Eigen::Array3f c(v.x(), v.y(), v.z());
            c.x() = c.x() * intensity;
            c.y() = c.y() * intensity;
            c.z() = c.z() * intensity + (1.f - intensity);
            c.matrix().normalize();
            o[12] = c.x(); o[13] = c.y(); o[14] = c.z();
        }
        return write_all(argv[3], out.data(), out.size() * sizeof(float)) ? 0 : 2;
    }
    if (mode == "order") {
        pcg32 rng;  // default state, as the camera's static Independent sampler (perspective.cpp:117-122)
        const Point2 p(rng.nextFloat(), rng.nextFloat());
        const float o[2] = {p.x, p.y};
        return write_all(argv[2], o, sizeof(o)) ? 0 : 2;
    }
    return 2;
}
