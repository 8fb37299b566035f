// Host image encoders (see image_io.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rr {

int encoder_threads();
bool encode_jpeg(const uint8_t* rgba, int W, int H, int quality, std::vector<uint8_t>& out, int threads = 0);
bool encode_png(const uint8_t* rgba, int W, int H, std::vector<uint8_t>& out, int level = 1);
bool write_file(const std::string& path, const std::vector<uint8_t>& data);

}  // namespace rr
