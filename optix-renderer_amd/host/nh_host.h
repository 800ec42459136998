// Internal declarations shared by the host-side translation units.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "nori_hip.h"

namespace nh {
void set_host_error(const std::string &msg);
// PNG -> 8-bit RGBA (png_decode.cpp); false with a message on malformed or unsupported files
bool png_decode_rgba8(const std::string &path, std::vector<uint8_t> &out, unsigned &width, unsigned &height,
                      std::string &err);
// Radiance RGBE .hdr -> float RGBA as the reference's HDRLoader decodes it (hdr_decode.cpp); false with a message on
// malformed or unsupported files
bool hdr_decode_rgba(const std::string &path, std::vector<float> &out, unsigned &width, unsigned &height,
                     std::string &err);
}
