// Minimal PNG decoder for texture ingestion (PNGTexture::loadFromFile, src/textures/PNGTexture.cpp:66-121,
// which decodes through lodepng to 8-bit RGBA). Written from the PNG specification (ISO/IEC 15948):
// chunk walk, zlib inflate of the concatenated IDAT stream, per-scanline unfiltering
// (None/Sub/Up/Average/Paeth), conversion of every non-interlaced colour type to RGBA8:
// grey and grey+alpha replicate the grey level, palette entries take tRNS alpha, a missing
// alpha channel is 255, 16-bit samples keep their high byte (what lodepng's RGBA8 output does).
// Adam7-interlaced files are rejected.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "nh_host.h"

namespace nh {

namespace {

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

}  // namespace

// 2^28 pixels: 1 GiB of RGBA8 output, at most 2 GiB of raw 64-bit scanlines (< 2^32 for zlib's uInt)
constexpr uint64_t kMaxPngPixels = (uint64_t)1 << 28;

bool png_decode_rgba8(const std::string &path, std::vector<uint8_t> &out, unsigned &width, unsigned &height,
                      std::string &err) {
    std::ifstream is(path, std::ios::binary);
    if (!is) return err = "cannot open " + path, false;
    std::vector<uint8_t> file((std::istreambuf_iterator<char>(is)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (file.size() < 8 || std::memcmp(file.data(), sig, 8) != 0) return err = path + ": not a PNG file", false;
    unsigned depth = 0, ctype = 0, interlace = 0;
    width = height = 0;
    std::vector<uint8_t> idat, palette, trns;
    bool seen_ihdr = false, seen_iend = false;
    for (size_t pos = 8; pos + 12 <= file.size() && !seen_iend;) {
        const uint32_t len = be32(&file[pos]);
        if (pos + 12 + (size_t)len > file.size()) return err = path + ": truncated chunk", false;
        const std::string type(reinterpret_cast<const char *>(&file[pos + 4]), 4);
        const uint8_t *data = &file[pos + 8];
        if (type == "IHDR") {
            if (len != 13) return err = path + ": bad IHDR", false;
            width = be32(data);
            height = be32(data + 4);
            depth = data[8];
            ctype = data[9];
            interlace = data[12];
            seen_ihdr = true;
        } else if (type == "PLTE") {
            palette.assign(data, data + len);
        } else if (type == "tRNS") {
            trns.assign(data, data + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), data, data + len);
        } else if (type == "IEND") {
            seen_iend = true;
        }
        pos += 12 + (size_t)len;
    }
    if (!seen_ihdr || width == 0 || height == 0) return err = path + ": missing IHDR", false;
    // the PNG spec limits each dimension to 2^31-1; the decoded RGBA8 image (and the 16-bit raw
    // scanlines, up to 8 bytes per pixel) must also fit the size_t / zlib uInt arithmetic below
    if (width > 0x7fffffffu || height > 0x7fffffffu || (uint64_t)width * height > kMaxPngPixels)
        return err = path + ": image too large", false;
    if (interlace != 0) return err = path + ": interlaced PNG is not supported", false;
    int channels;
    switch (ctype) {
        case 0: channels = 1; break;  // grey
        case 2: channels = 3; break;  // RGB
        case 3: channels = 1; break;  // palette
        case 4: channels = 2; break;  // grey + alpha
        case 6: channels = 4; break;  // RGBA
        default: return err = path + ": bad colour type", false;
    }
    const bool depth_ok = (ctype == 3) ? (depth == 1 || depth == 2 || depth == 4 || depth == 8)
                          : (ctype == 0) ? (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)
                                         : (depth == 8 || depth == 16);
    if (!depth_ok) return err = path + ": unsupported bit depth", false;
    if (ctype == 3 && palette.empty()) return err = path + ": palette image without PLTE", false;
    const size_t bits_pp = (size_t)channels * depth;
    const size_t stride = ((size_t)width * bits_pp + 7) / 8;
    const size_t bpp = std::max<size_t>(1, bits_pp / 8);  // filter byte distance
    std::vector<uint8_t> raw((stride + 1) * (size_t)height);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) return err = "zlib init failed", false;
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if (zr != Z_STREAM_END || zs.total_out != raw.size()) return err = path + ": corrupt image data", false;
    // unfilter in place
    std::vector<uint8_t> prev(stride, 0);
    for (unsigned y = 0; y < height; ++y) {
        uint8_t *row = &raw[(size_t)y * (stride + 1)];
        const uint8_t f = row[0];
        uint8_t *cur = row + 1;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
            int v = cur[i];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: return err = path + ": bad filter type", false;
            }
            cur[i] = (uint8_t)v;
        }
        std::memcpy(prev.data(), cur, stride);
    }
    // convert to RGBA8
    out.assign((size_t)width * height * 4, 255);
    for (unsigned y = 0; y < height; ++y) {
        const uint8_t *row = &raw[(size_t)y * (stride + 1) + 1];
        for (unsigned x = 0; x < width; ++x) {
            uint8_t *o = &out[((size_t)y * width + x) * 4];
            auto sample = [&](int ch) -> unsigned {  // one channel, 8-bit (16-bit: high byte)
                if (depth >= 8) return row[((size_t)x * channels + ch) * (depth / 8)];
                const size_t bit = (size_t)x * depth;
                return (row[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
            };
            if (ctype == 3) {
                const unsigned idx = sample(0);
                if ((size_t)idx * 3 + 2 >= palette.size()) return err = path + ": palette index out of range", false;
                o[0] = palette[3 * idx];
                o[1] = palette[3 * idx + 1];
                o[2] = palette[3 * idx + 2];
                o[3] = idx < trns.size() ? trns[idx] : 255;
            } else if (ctype == 0 || ctype == 4) {
                unsigned g = sample(0);
                if (depth < 8) g = g * 255 / ((1u << depth) - 1);
                o[0] = o[1] = o[2] = (uint8_t)g;
                if (ctype == 4) o[3] = (uint8_t)sample(1);
            } else {
                o[0] = (uint8_t)sample(0);
                o[1] = (uint8_t)sample(1);
                o[2] = (uint8_t)sample(2);
                if (ctype == 6) o[3] = (uint8_t)sample(3);
            }
        }
    }
    return true;
}

}  // namespace nh
