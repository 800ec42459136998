// TEST INFRASTRUCTURE ONLY. Radiance .hdr probe: compiled by oracle/build_ref.sh against the reference's own decoder
// (/root/reference/include/nori/HDRLoader.h, a self-contained header: <math.h>, <memory.h>, <stdio.h>), unmodified,
// with the reference's floating-point setup (x86-64 SSE2, no FMA contraction). It runs HDRLoader::load -- what
// PNGTexture::loadFromFile calls for a .hdr file (PNGTexture.cpp:97-117) -- and writes the texels, so
// tests/test_hdr.py can pin the product decoder (host/hdr_decode.cpp) against the reference's own on well-formed
// files of every encoding (the reference reads malformed files into undefined memory; those are not compared).
//
// usage: hdr_probe IN.hdr OUT   OUT = int32 width, int32 height, then width * height * 4 floats (HDRLoaderResult::cols)
#include <nori/HDRLoader.h>

#include <cstdint>
#include <cstdio>

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    nori::HDRLoader::HDRLoaderResult res{};
    if (!nori::HDRLoader::load(argv[1], res)) return 3;
    FILE *f = std::fopen(argv[2], "wb");
    if (!f) return 2;
    const int32_t wh[2] = {res.width, res.height};
    bool ok = std::fwrite(wh, sizeof(wh), 1, f) == 1;
    const size_t n = (size_t)res.width * (size_t)res.height * 4;
    ok = ok && std::fwrite(res.cols, sizeof(float), n, f) == n;
    delete[] res.cols;
    return std::fclose(f) == 0 && ok ? 0 : 2;
}
