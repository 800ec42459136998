// Radiance RGBE (.hdr) images as PNGTexture::loadFromFile's ".hdr" branch reads them (src/textures/PNGTexture.cpp:97-117)
// through the reference's HDRLoader (include/nori/HDRLoader.h, after flipcode's HDR_Image_Reader): a "#?RADIANCE"
// signature, header lines up to an empty line, a "-Y h +X w" resolution line, then h scanlines of w RGBE pixels --
// new-style run-length scanlines (2, 2, hi, lo, then each component's runs) for 8 <= w <= 0x7fff, otherwise (or when
// the scanline does not start that way) flat RGBE pixels with the old (1, 1, 1, n) repeat codes. Scanlines land in
// file order (row 0 = the first one); a pixel is (m / 256.0f) * (float)pow(2, e - 128) per channel, alpha 0
// (HDRLoader.h:27-44). No gamma: the floats are used as they are.
//
// The reference reads without bounds checks (runs past a scanline, a repeat before the first pixel, a truncated file
// leave memory or rows undefined); here every such file is an error, so only well-formed files load -- and those
// decode to the reference's floats (tests/test_textures.py: a numpy restatement on synthetic files of every encoding).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "nh_host.h"

namespace nh {
namespace {

constexpr int kMinLen = 8, kMaxLen = 0x7fff;
constexpr uint64_t kMaxHdrPixels = (uint64_t)1 << 28;

struct Reader {
    const std::vector<uint8_t> &b;
    size_t pos = 0;
    bool eof = false;  // a read past the end (fgetc's EOF; feof after it)
    int get() {
        if (pos >= b.size()) {
            eof = true;
            return -1;
        }
        return b[pos++];
    }
};

// HDRLoader.h oldDecrunch: flat RGBE pixels; (1, 1, 1, n) repeats the previous pixel n << rshift times
bool old_decrunch(Reader &r, uint8_t (*line)[4], int first, int len, std::string &err) {
    int rshift = 0, x = first;
    while (len > 0) {
        uint8_t p[4];
        for (int c = 0; c < 4; ++c) p[c] = (uint8_t)r.get();
        if (r.eof) return err = "truncated scanline", false;
        if (p[0] == 1 && p[1] == 1 && p[2] == 1) {
            if (x == 0) return err = "repeat code before the first pixel of a scanline", false;
            // the count p[3] << rshift, checked against the scanline's rest before it is formed: chained repeat codes
            // grow rshift by 8 each, and the reference's int shift overflows (undefined) from rshift 24 on
            if (p[3] != 0 && (rshift > 24 || ((uint64_t)p[3] << rshift) > (uint64_t)len))
                return err = "repeat code past the end of a scanline", false;
            for (uint64_t i = p[3] == 0 ? 0 : (uint64_t)p[3] << rshift; i > 0; --i) {
                std::memcpy(line[x], line[x - 1], 4);
                ++x;
                --len;
            }
            rshift += 8;
            if (rshift > 64) rshift = 64;  // (zero-count codes may chain without bound)
        } else {
            std::memcpy(line[x], p, 4);
            ++x;
            --len;
            rshift = 0;
        }
    }
    return true;
}

// HDRLoader.h decrunch: one scanline of w pixels
bool decrunch(Reader &r, uint8_t (*line)[4], int w, std::string &err) {
    if (w < kMinLen || w > kMaxLen) return old_decrunch(r, line, 0, w, err);
    const int i0 = r.get();
    if (i0 != 2) {
        if (!r.eof) --r.pos;  // fseek(file, -1, SEEK_CUR)
        r.eof = false;
        return old_decrunch(r, line, 0, w, err);
    }
    line[0][1] = (uint8_t)r.get();
    line[0][2] = (uint8_t)r.get();
    const int i = r.get();
    if (line[0][1] != 2 || (line[0][2] & 128)) {
        line[0][0] = 2;
        line[0][3] = (uint8_t)i;
        if (r.eof) return err = "truncated scanline", false;
        return old_decrunch(r, line, 1, w - 1, err);
    }
    for (int c = 0; c < 4; ++c)
        for (int j = 0; j < w;) {
            int code = r.get();
            if (r.eof) return err = "truncated scanline", false;
            if (code > 128) {  // run
                code &= 127;
                const uint8_t v = (uint8_t)r.get();
                if (j + code > w) return err = "run past the end of a scanline", false;
                while (code--) line[j++][c] = v;
            } else {  // literal bytes
                if (j + code > w) return err = "run past the end of a scanline", false;
                while (code--) line[j++][c] = (uint8_t)r.get();
            }
        }
    if (r.eof) return err = "truncated scanline", false;
    return true;
}

// HDRLoader.h convertComponent: v = val / 256.0f, d = (float)pow(2, expo), v * d
float component(int expo, int val) {
    const float v = (float)val / 256.0f;
    const float d = (float)std::pow(2.0, (double)expo);
    return v * d;
}

}  // namespace

bool hdr_decode_rgba(const std::string &path, std::vector<float> &out, unsigned &width, unsigned &height,
                     std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return err = "cannot open " + path, false;
    const std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    Reader r{bytes};
    if (bytes.size() < 11 || std::memcmp(bytes.data(), "#?RADIANCE", 10) != 0)
        return err = "not a Radiance HDR file", false;
    r.pos = 11;  // the signature and the byte after it (fseek(file, 1, SEEK_CUR))
    // header lines, up to two consecutive newlines
    for (int c = 0, oldc; ;) {
        oldc = c;
        c = r.get();
        if (r.eof) return err = "truncated header", false;
        if (c == 0xa && oldc == 0xa) break;
    }
    std::string reso;
    for (;;) {
        const int c = r.get();
        if (r.eof) return err = "truncated resolution line", false;
        reso.push_back((char)c);
        if (c == 0xa) break;
        if (reso.size() > 200) return err = "resolution line too long", false;
    }
    int w = 0, h = 0;
    if (std::sscanf(reso.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0)
        return err = "unsupported resolution line (only -Y h +X w): " + reso, false;
    if ((uint64_t)w * (uint64_t)h > kMaxHdrPixels) return err = "image too large", false;
    width = (unsigned)w;
    height = (unsigned)h;
    out.assign(4 * (size_t)w * h, 0.f);
    std::vector<uint8_t> line(4 * (size_t)w);
    auto *ln = reinterpret_cast<uint8_t (*)[4]>(line.data());
    for (int y = 0; y < h; ++y) {
        if (!decrunch(r, ln, w, err)) return err = "scanline " + std::to_string(y) + ": " + err, false;
        float *row = &out[4 * (size_t)y * w];
        for (int x = 0; x < w; ++x) {
            const int expo = (int)ln[x][3] - 128;
            row[4 * x] = component(expo, ln[x][0]);
            row[4 * x + 1] = component(expo, ln[x][1]);
            row[4 * x + 2] = component(expo, ln[x][2]);
            row[4 * x + 3] = 0.f;
        }
    }
    return true;
}

}  // namespace nh
