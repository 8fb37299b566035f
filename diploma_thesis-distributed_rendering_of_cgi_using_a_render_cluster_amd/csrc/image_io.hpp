// Host image encoders (see image_io.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rr {

int encoder_threads();

// Baseline JPEG tables for a quality: quantisers (natural order), their
// reciprocals, and the 8x8 DCT basis c[u][x] = C(u)/2 cos((2x+1) u pi / 16).
struct JpegTables {
    uint8_t ql[64], qc[64];
    float qinv_l[64], qinv_c[64];
    float dct[64];
};
void jpeg_tables(int quality, JpegTables& t);
// Quantised coefficients of a whole image: [mcuy][mcux][6 blocks][64], natural
// order, blocks Y00 Y01 Y10 Y11 Cb Cr (4:2:0, edge-replicated padding).
size_t jpeg_coeff_count(int W, int H);
bool encode_jpeg_coeffs(const int16_t* coeffs, int W, int H, int quality, std::vector<uint8_t>& out,
                        int threads = 0);
// The file bytes in front of the entropy-coded segment (SOI ... SOS), and the
// Huffman tables as 4 x 256 packed code | len << 16 (DC luma, AC luma, DC
// chroma, AC chroma) for the device coder (jpeg.hip).
void jpeg_header_bytes(int W, int H, int quality, std::vector<uint8_t>& out);
void jpeg_huff_tables(uint32_t out[4 * 256]);
bool encode_jpeg(const uint8_t* rgba, int W, int H, int quality, std::vector<uint8_t>& out, int threads = 0);
bool encode_png(const uint8_t* rgba, int W, int H, std::vector<uint8_t>& out, int level = 1, int threads = 0);
bool write_file(const std::string& path, const std::vector<uint8_t>& data);

}  // namespace rr
