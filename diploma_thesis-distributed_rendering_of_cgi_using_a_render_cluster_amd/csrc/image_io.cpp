// Host image encoders: baseline JPEG (JFIF, 4:2:0, ITU T.81 Annex K tables,
// IJG quality scaling) and PNG (zlib). Replaces Blender's write_still for the
// formats the reference jobs use: "JPEG" with quality forced to 90
// (/root/reference/scripts/render-timing-script.py:83-84) and "PNG"
// (blender-projects/02_physics/02-physics_demo_170f-5w_naive-fine.toml:13).
//
// The JPEG entropy coder runs one restart interval per MCU row, so rows are
// encoded on parallel host threads and joined with RSTn markers.
#include "image_io.hpp"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>

#include <sched.h>

namespace rr {

// Host threads of the encoders: the CPUs this process may run on (a worker
// pinned to its GPU's NUMA node — bench.py gpu_placement — gets that share,
// not the machine's count), at most 16.
int encoder_threads() {
    int n = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (n <= 0) n = 4;
    return std::min(n, 16);
}

namespace {

// ---------------------------------------------------------------- JPEG ----
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

const uint8_t kStdLuma[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                              14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                              18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                              49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kStdChroma[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// Annex K.3 Huffman tables: BITS (16) + HUFFVAL.
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct HuffTable {
    uint16_t code[256];
    uint8_t len[256];
    void build(const uint8_t bits[16], const uint8_t* vals) {
        std::memset(len, 0, sizeof len);
        uint16_t c = 0;
        int k = 0;
        for (int l = 1; l <= 16; ++l) {
            for (int i = 0; i < bits[l - 1]; ++i) {
                code[vals[k]] = c++;
                len[vals[k]] = (uint8_t)l;
                ++k;
            }
            c <<= 1;
        }
    }
};

struct Tables {
    HuffTable dc[2], ac[2];
    Tables() {
        dc[0].build(kDcLumBits, kDcLumVal);
        dc[1].build(kDcChrBits, kDcChrVal);
        ac[0].build(kAcLumBits, kAcLumVal);
        ac[1].build(kAcChrBits, kAcChrVal);
    }
};
const Tables& tables() {
    static Tables t;
    return t;
}

struct BitWriter {
    std::vector<uint8_t>& out;
    uint32_t acc = 0;
    int nbits = 0;
    explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
    inline void put(uint32_t code, int len) {
        acc = (acc << len) | (code & ((1u << len) - 1u));
        nbits += len;
        while (nbits >= 8) {
            const uint8_t b = (uint8_t)(acc >> (nbits - 8));
            out.push_back(b);
            if (b == 0xFF) out.push_back(0x00);
            nbits -= 8;
        }
        acc &= (1u << nbits) - 1u;
    }
    void flush() {  // pad with 1-bits
        if (nbits > 0) put((1u << (8 - nbits)) - 1u, 8 - nbits);
    }
};

// IJG jpeg_quality_scaling + jpeg_add_quant_table (force_baseline).
void quant_table(const uint8_t* base, int quality, uint8_t* q) {
    quality = std::min(std::max(quality, 1), 100);
    const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
    for (int i = 0; i < 64; ++i) {
        long t = ((long)base[i] * scale + 50L) / 100L;
        if (t <= 0) t = 1;
        if (t > 255) t = 255;
        q[i] = (uint8_t)t;
    }
}

struct Dct {
    float c[8][8];  // c[u][x] = C(u)/2 cos((2x+1) u pi / 16)
    Dct() {
        for (int u = 0; u < 8; ++u)
            for (int x = 0; x < 8; ++x)
                c[u][x] = (float)((u == 0 ? std::sqrt(0.5) : 1.0) * 0.5 * std::cos((2 * x + 1) * u * M_PI / 16.0));
    }
};
const Dct& dct() {
    static Dct d;
    return d;
}

// Forward DCT + quantisation of one 8x8 block (level-shifted samples).
void fdct_quant(const float in[64], const float qinv[64], int16_t* out) {
    const Dct& D = dct();
    float tmp[64];
    for (int y = 0; y < 8; ++y)
        for (int u = 0; u < 8; ++u) {
            float s = 0.f;
            for (int x = 0; x < 8; ++x) s += D.c[u][x] * in[8 * y + x];
            tmp[8 * y + u] = s;
        }
    for (int v = 0; v < 8; ++v)
        for (int u = 0; u < 8; ++u) {
            float s = 0.f;
            for (int y = 0; y < 8; ++y) s += D.c[v][y] * tmp[8 * y + u];
            out[8 * v + u] = (int16_t)std::lrint(s * qinv[8 * v + u]);
        }
}

inline int bitlen(int v) {
    v = v < 0 ? -v : v;
    int n = 0;
    while (v) { ++n; v >>= 1; }
    return n;
}

void encode_block(BitWriter& bw, const int16_t* blk, int& pred, const HuffTable& dc, const HuffTable& ac) {
    const int diff = blk[0] - pred;
    pred = blk[0];
    int n = bitlen(diff);
    bw.put(dc.code[n], dc.len[n]);
    if (n) bw.put(diff < 0 ? (uint32_t)(diff - 1) : (uint32_t)diff, n);
    int run = 0;
    for (int k = 1; k < 64; ++k) {
        const int v = blk[kZigzag[k]];
        if (v == 0) {
            ++run;
            continue;
        }
        while (run > 15) {
            bw.put(ac.code[0xF0], ac.len[0xF0]);
            run -= 16;
        }
        n = bitlen(v);
        const int sym = (run << 4) | n;
        bw.put(ac.code[sym], ac.len[sym]);
        bw.put(v < 0 ? (uint32_t)(v - 1) : (uint32_t)v, n);
        run = 0;
    }
    if (run) bw.put(ac.code[0x00], ac.len[0x00]);
}

void put16(std::vector<uint8_t>& o, int v) {
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void write_dht(std::vector<uint8_t>& o, int cls, int id, const uint8_t bits[16], const uint8_t* vals) {
    int n = 0;
    for (int i = 0; i < 16; ++i) n += bits[i];
    o.push_back(0xFF); o.push_back(0xC4);
    put16(o, 2 + 1 + 16 + n);
    o.push_back((uint8_t)((cls << 4) | id));
    o.insert(o.end(), bits, bits + 16);
    o.insert(o.end(), vals, vals + n);
}

// Forward DCT + quantisation of MCU row `my` (16 pixel rows) on the host:
// coefficients [mcux][6][64] (blocks Y00 Y01 Y10 Y11 Cb Cr, natural order).
// jpeg.hip computes the same values on the device with the same float ops.
void mcu_row_coeffs(const uint8_t* rgba, int W, int H, int my, const float qy[64], const float qc[64],
                    int16_t* out) {
    const int mcux = (W + 15) / 16;
    float Y[4][64], Cb[64], Cr[64];
    for (int mx = 0; mx < mcux; ++mx) {
        float cbs[16][16], crs[16][16];
        for (int yy = 0; yy < 16; ++yy) {
            const int sy = std::min(my * 16 + yy, H - 1);
            for (int xx = 0; xx < 16; ++xx) {
                const int sx = std::min(mx * 16 + xx, W - 1);
                const uint8_t* p = rgba + 4 * ((size_t)sy * W + sx);
                const float r = p[0], g = p[1], b = p[2];
                const float y = 0.299f * r + 0.587f * g + 0.114f * b;
                Y[(yy >> 3) * 2 + (xx >> 3)][8 * (yy & 7) + (xx & 7)] = y - 128.0f;
                cbs[yy][xx] = -0.168735892f * r - 0.331264108f * g + 0.5f * b;
                crs[yy][xx] = 0.5f * r - 0.418687589f * g - 0.081312411f * b;
            }
        }
        for (int yy = 0; yy < 8; ++yy)
            for (int xx = 0; xx < 8; ++xx) {
                Cb[8 * yy + xx] = 0.25f * (cbs[2 * yy][2 * xx] + cbs[2 * yy][2 * xx + 1] + cbs[2 * yy + 1][2 * xx] +
                                           cbs[2 * yy + 1][2 * xx + 1]);
                Cr[8 * yy + xx] = 0.25f * (crs[2 * yy][2 * xx] + crs[2 * yy][2 * xx + 1] + crs[2 * yy + 1][2 * xx] +
                                           crs[2 * yy + 1][2 * xx + 1]);
            }
        int16_t* o = out + (size_t)mx * 6 * 64;
        for (int k = 0; k < 4; ++k) fdct_quant(Y[k], qy, o + 64 * k);
        fdct_quant(Cb, qc, o + 64 * 4);
        fdct_quant(Cr, qc, o + 64 * 5);
    }
}

// Huffman-code one MCU row (one restart interval) from its coefficients.
void entropy_mcu_row(const int16_t* coeffs, int mcux, std::vector<uint8_t>& out) {
    const Tables& T = tables();
    BitWriter bw(out);
    int pred[3] = {0, 0, 0};
    for (int mx = 0; mx < mcux; ++mx) {
        const int16_t* o = coeffs + (size_t)mx * 6 * 64;
        for (int k = 0; k < 4; ++k) encode_block(bw, o + 64 * k, pred[0], T.dc[0], T.ac[0]);
        encode_block(bw, o + 64 * 4, pred[1], T.dc[1], T.ac[1]);
        encode_block(bw, o + 64 * 5, pred[2], T.dc[1], T.ac[1]);
    }
    bw.flush();
}

void jpeg_header(int W, int H, const uint8_t* ql, const uint8_t* qc, std::vector<uint8_t>& out) {
    // SOI + APP0 JFIF
    const uint8_t soi_app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,
                                0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    out.insert(out.end(), soi_app0, soi_app0 + sizeof soi_app0);
    // DQT (tables in zigzag order)
    for (int t = 0; t < 2; ++t) {
        const uint8_t* q = t ? qc : ql;
        out.push_back(0xFF); out.push_back(0xDB);
        put16(out, 67);
        out.push_back((uint8_t)t);
        for (int k = 0; k < 64; ++k) out.push_back(q[kZigzag[k]]);
    }
    // SOF0: 3 components, Y 2x2, Cb/Cr 1x1
    out.push_back(0xFF); out.push_back(0xC0);
    put16(out, 17);
    out.push_back(8);
    put16(out, H);
    put16(out, W);
    out.push_back(3);
    const uint8_t comps[9] = {1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1};
    out.insert(out.end(), comps, comps + 9);
    write_dht(out, 0, 0, kDcLumBits, kDcLumVal);
    write_dht(out, 1, 0, kAcLumBits, kAcLumVal);
    write_dht(out, 0, 1, kDcChrBits, kDcChrVal);
    write_dht(out, 1, 1, kAcChrBits, kAcChrVal);
    // DRI: one restart interval per MCU row
    out.push_back(0xFF); out.push_back(0xDD);
    put16(out, 4);
    put16(out, (W + 15) / 16);
    // SOS
    const uint8_t sos[] = {0xFF, 0xDA, 0x00, 0x0C, 0x03, 1, 0x00, 2, 0x11, 3, 0x11, 0x00, 0x3F, 0x00};
    out.insert(out.end(), sos, sos + sizeof sos);
}

// Run fn(my) for every MCU row on `threads` host threads.
template <typename Fn>
void for_rows(int mcuy, int threads, Fn fn) {
    if (threads <= 0) threads = encoder_threads();
    threads = std::max(1, std::min(threads, mcuy));
    if (threads == 1) {
        for (int my = 0; my < mcuy; ++my) fn(my);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            for (int my = t; my < mcuy; my += threads) fn(my);
        });
    for (auto& th : pool) th.join();
}

void join_rows(std::vector<std::vector<uint8_t>>& rows, std::vector<uint8_t>& out) {
    const int mcuy = (int)rows.size();
    for (int my = 0; my < mcuy; ++my) {
        out.insert(out.end(), rows[my].begin(), rows[my].end());
        if (my + 1 < mcuy) {
            out.push_back(0xFF);
            out.push_back((uint8_t)(0xD0 + (my & 7)));
        }
    }
    out.push_back(0xFF); out.push_back(0xD9);
}

// --------------------------------------------------------------- PNG ------
void png_chunk(std::vector<uint8_t>& o, const char* type, const uint8_t* data, size_t n) {
    const uint32_t len = (uint32_t)n;
    o.push_back((uint8_t)(len >> 24)); o.push_back((uint8_t)(len >> 16));
    o.push_back((uint8_t)(len >> 8)); o.push_back((uint8_t)len);
    const size_t start = o.size();
    o.insert(o.end(), type, type + 4);
    if (n) o.insert(o.end(), data, data + n);
    const uint32_t crc = (uint32_t)crc32(0L, o.data() + start, (uInt)(o.size() - start));
    o.push_back((uint8_t)(crc >> 24)); o.push_back((uint8_t)(crc >> 16));
    o.push_back((uint8_t)(crc >> 8)); o.push_back((uint8_t)crc);
}

}  // namespace

void jpeg_tables(int quality, JpegTables& t) {
    quant_table(kStdLuma, quality, t.ql);
    quant_table(kStdChroma, quality, t.qc);
    for (int i = 0; i < 64; ++i) {  // quantisation folded as a multiply by 1/q
        t.dct[i] = dct().c[i / 8][i % 8];
        t.qinv_l[i] = 1.0f / (float)t.ql[i];
        t.qinv_c[i] = 1.0f / (float)t.qc[i];
    }
}

void jpeg_header_bytes(int W, int H, int quality, std::vector<uint8_t>& out) {
    JpegTables t;
    jpeg_tables(quality, t);
    out.clear();
    jpeg_header(W, H, t.ql, t.qc, out);
}

void jpeg_huff_tables(uint32_t out[4 * 256]) {
    const Tables& T = tables();
    const HuffTable* order[4] = {&T.dc[0], &T.ac[0], &T.dc[1], &T.ac[1]};
    for (int t = 0; t < 4; ++t)
        for (int s = 0; s < 256; ++s) out[256 * t + s] = (uint32_t)order[t]->code[s] | ((uint32_t)order[t]->len[s] << 16);
}

size_t jpeg_coeff_count(int W, int H) { return (size_t)((W + 15) / 16) * ((H + 15) / 16) * 6 * 64; }

bool encode_jpeg(const uint8_t* rgba, int W, int H, int quality, std::vector<uint8_t>& out, int threads) {
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535) return false;
    JpegTables t;
    jpeg_tables(quality, t);
    const int mcux = (W + 15) / 16, mcuy = (H + 15) / 16;
    out.clear();
    out.reserve((size_t)W * H / 2);
    jpeg_header(W, H, t.ql, t.qc, out);
    std::vector<std::vector<uint8_t>> rows((size_t)mcuy);
    for_rows(mcuy, threads, [&](int my) {
        std::vector<int16_t> c((size_t)mcux * 6 * 64);
        mcu_row_coeffs(rgba, W, H, my, t.qinv_l, t.qinv_c, c.data());
        rows[my].reserve((size_t)mcux * 256);
        entropy_mcu_row(c.data(), mcux, rows[my]);
    });
    join_rows(rows, out);
    return true;
}

bool encode_jpeg_coeffs(const int16_t* coeffs, int W, int H, int quality, std::vector<uint8_t>& out,
                        int threads) {
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535) return false;
    JpegTables t;
    jpeg_tables(quality, t);
    const int mcux = (W + 15) / 16, mcuy = (H + 15) / 16;
    out.clear();
    out.reserve((size_t)W * H / 2);
    jpeg_header(W, H, t.ql, t.qc, out);
    std::vector<std::vector<uint8_t>> rows((size_t)mcuy);
    for_rows(mcuy, threads, [&](int my) {
        rows[my].reserve((size_t)mcux * 256);
        entropy_mcu_row(coeffs + (size_t)my * mcux * 6 * 64, mcux, rows[my]);
    });
    join_rows(rows, out);
    return true;
}

// PNG (8-bit RGBA, filter Sub on every row). The zlib stream is deflated in
// bands of rows on host threads, pigz-style: each band is a raw deflate stream
// ended with a sync flush (an empty stored block, byte-aligned), the last one
// with the final block; concatenated they form one deflate stream, wrapped in
// the zlib header and the Adler-32 of the whole image (adler32_combine of the
// bands'). A band restarts the 32 KB match window, which costs a little ratio
// and no correctness. A 1080p 02 frame: one thread took most of the frame's
// time on the host, more than the GPU's.
bool encode_png(const uint8_t* rgba, int W, int H, std::vector<uint8_t>& out, int level, int threads) {
    if (W <= 0 || H <= 0) return false;
    const size_t stride = (size_t)W * 4;
    std::vector<uint8_t> raw((stride + 1) * H);
    if (threads <= 0) threads = encoder_threads();
    const int bands = std::max(1, std::min(threads, H / 16));  // >= 16 rows a band
    std::vector<std::vector<uint8_t>> zb(bands);
    std::vector<uLong> adl(bands), len(bands);
    std::vector<int> ok(bands, 0);
    auto band = [&](int b) {
        const int y0 = (int)((long)H * b / bands), y1 = (int)((long)H * (b + 1) / bands);
        for (int y = y0; y < y1; ++y) {
            uint8_t* dst = &raw[(stride + 1) * y];
            const uint8_t* src = rgba + stride * y;
            dst[0] = 1;
            for (size_t x = 0; x < stride; ++x) dst[1 + x] = (uint8_t)(src[x] - (x >= 4 ? src[x - 4] : 0));
        }
        const uint8_t* in = &raw[(stride + 1) * y0];
        const uLong n = (uLong)((stride + 1) * (size_t)(y1 - y0));
        z_stream zs{};
        if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return;
        zb[b].resize(deflateBound(&zs, n) + 16);
        zs.next_in = const_cast<Bytef*>(in);
        zs.avail_in = (uInt)n;
        zs.next_out = zb[b].data();
        zs.avail_out = (uInt)zb[b].size();
        const int rc = deflate(&zs, b == bands - 1 ? Z_FINISH : Z_SYNC_FLUSH);
        const bool done = b == bands - 1 ? rc == Z_STREAM_END : (rc == Z_OK && zs.avail_in == 0);
        zb[b].resize(zb[b].size() - zs.avail_out);
        deflateEnd(&zs);
        adl[b] = adler32(adler32(0L, Z_NULL, 0), in, (uInt)n);
        len[b] = n;
        ok[b] = done ? 1 : 0;
    };
    if (bands == 1) {
        band(0);
    } else {
        std::vector<std::thread> pool;
        for (int b = 0; b < bands; ++b) pool.emplace_back(band, b);
        for (auto& t : pool) t.join();
    }
    std::vector<uint8_t> z = {0x78, 0x01};  // zlib header: deflate, 32 KB window, no dictionary
    uLong a = adler32(0L, Z_NULL, 0);
    for (int b = 0; b < bands; ++b) {
        if (!ok[b]) return false;
        z.insert(z.end(), zb[b].begin(), zb[b].end());
        a = adler32_combine(a, adl[b], (z_off_t)len[b]);
    }
    for (int k = 3; k >= 0; --k) z.push_back((uint8_t)(a >> (8 * k)));
    out.clear();
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    out.insert(out.end(), sig, sig + 8);
    uint8_t ihdr[13] = {(uint8_t)(W >> 24), (uint8_t)(W >> 16), (uint8_t)(W >> 8), (uint8_t)W,
                        (uint8_t)(H >> 24), (uint8_t)(H >> 16), (uint8_t)(H >> 8), (uint8_t)H,
                        8, 6, 0, 0, 0};
    png_chunk(out, "IHDR", ihdr, 13);
    png_chunk(out, "IDAT", z.data(), z.size());
    png_chunk(out, "IEND", nullptr, 0);
    return true;
}

bool write_file(const std::string& path, const std::vector<uint8_t>& data) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const size_t n = std::fwrite(data.data(), 1, data.size(), f);
    const bool ok = n == data.size() && std::fclose(f) == 0;
    if (n != data.size()) std::fclose(f);
    return ok;
}

}  // namespace rr
