// JPEG forward transform on the device: RGB -> YCbCr (JFIF), 4:2:0 chroma
// averaging, 8x8 forward DCT and quantisation of the tonemapped frame, so only
// Huffman coding (image_io.cpp, one restart interval per MCU row on host
// threads) stays on the CPU and 6 blocks x 64 int16 per 16x16 MCU cross PCIe.
// Same float ops in the same order as image_io.cpp's mcu_row_coeffs /
// fdct_quant (no contraction), so the file bytes equal the host encoder's.
// Replaces the JPEG side of Blender's write_still (render-timing-script.py:83-84).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "device.hpp"

namespace rr {

namespace {

__constant__ uint8_t c_zigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                     12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                     35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                     58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// One 64-thread workgroup per 8x8 block; blocks 0..3 = Y (2x2), 4 = Cb, 5 = Cr.
// tab: dct[64] | qinv_luma[64] | qinv_chroma[64].
// Returns this lane's quantised coefficient (natural position threadIdx.x).
__device__ __forceinline__ int fdct_block(const uchar4* __restrict__ rgba, int W, int H, int mcux,
                                          const float* __restrict__ tab, int16_t* __restrict__ out, int blk) {
    __shared__ float in[64];
    __shared__ float tmp[64];
    const int mcu = blockIdx.x / 6;
    const int mx = mcu % mcux, my = mcu / mcux;
    const int t = threadIdx.x;
    const int ty = t >> 3, tx = t & 7;
    if (blk < 4) {
        const int sy = min(my * 16 + (blk >> 1) * 8 + ty, H - 1);
        const int sx = min(mx * 16 + (blk & 1) * 8 + tx, W - 1);
        const uchar4 p = rgba[(size_t)sy * W + sx];
        const float r = p.x, g = p.y, b = p.z;
        const float y = 0.299f * r + 0.587f * g + 0.114f * b;
        in[t] = y - 128.0f;
    } else {
        float v[4];
        for (int k = 0; k < 4; ++k) {
            const int sy = min(my * 16 + 2 * ty + (k >> 1), H - 1);
            const int sx = min(mx * 16 + 2 * tx + (k & 1), W - 1);
            const uchar4 p = rgba[(size_t)sy * W + sx];
            const float r = p.x, g = p.y, b = p.z;
            v[k] = blk == 4 ? -0.168735892f * r - 0.331264108f * g + 0.5f * b
                            : 0.5f * r - 0.418687589f * g - 0.081312411f * b;
        }
        in[t] = 0.25f * (v[0] + v[1] + v[2] + v[3]);
    }
    __syncthreads();
    {  // rows: tmp[y][u] = sum_x c[u][x] * in[y][x]
        const int y = ty, u = tx;
        float s = 0.f;
        for (int x = 0; x < 8; ++x) s += tab[8 * u + x] * in[8 * y + x];
        tmp[8 * y + u] = s;
    }
    __syncthreads();
    {  // columns: out[v][u] = sum_y c[v][y] * tmp[y][u], then quantise
        const int v = ty, u = tx;
        float s = 0.f;
        for (int y = 0; y < 8; ++y) s += tab[8 * v + y] * tmp[8 * y + u];
        const float* qinv = tab + (blk < 4 ? 64 : 128);
        const int16_t q = (int16_t)rintf(s * qinv[8 * v + u]);
        out[((size_t)mcu * 6 + blk) * 64 + 8 * v + u] = q;
        return q;
    }
}

// ------------------------------------------------------ entropy coding ---
// Baseline Huffman coding of the quantised coefficients on the device, byte for
// byte the host coder's output (image_io.cpp entropy_mcu_row + join_rows): one
// restart interval per MCU row, DC prediction reset per row, 1-bit padding,
// 0xFF stuffing, RSTn between rows, EOI. Only the entropy-coded bytes (~0.2-0.5
// MB for a 1080p frame at q90) cross PCIe instead of 6.2 MB of coefficients.
//
// One wave per 8x8 block, lane k = zigzag position k (the JPEG symbol order):
//  - k_jpeg_fdct_bits: the forward transform above + the block's AC bit count
//    (run lengths from a ballot of the nonzero lanes);
//  - k_jpeg_scan (workgroup per MCU row): + DC bits (prediction from the
//    previous block of the component), exclusive scan -> block bit offsets,
//    zeroes the row's words;
//  - k_jpeg_emit: every lane ORs its symbols (ZRLs, code, magnitude; DC on
//    lane 0, EOB after lane 63) into the row's MSB-first 32-bit words at its
//    scanned bit offset;
//  - k_jpeg_finish (workgroup per row): 1-bit padding, byte stuffing;
//  - k_jpeg_gather: rows at the prefix of their lengths with RSTn / EOI;
//  - k_jpeg_to_host: the stream into pinned host memory with 16-byte stores.
constexpr int kJpegThreads = 256;

__device__ __forceinline__ int cat_bits(int v) {  // JPEG magnitude category (bit length of |v|)
    v = v < 0 ? -v : v;
    return v ? 32 - __clz(v) : 0;
}
__device__ __forceinline__ uint32_t mag_bits(int v, int n) {  // the n magnitude bits of v
    return (v < 0 ? (uint32_t)(v - 1) : (uint32_t)v) & ((1u << n) - 1u);
}

// huff[t * 256 + sym] = code | len << 16; t: 0 DC luma, 1 AC luma, 2 DC chroma, 3 AC chroma.
// Lane k >= 1 of a block's wave: its AC symbols (ZRLs + run/size code +
// magnitude) as a bit string, MSB-aligned in a 64-bit word; returns the length.
// Lane 63 also carries the EOB when the block ends in zeros.
__device__ __forceinline__ int ac_lane(int v, int k, uint64_t nz, const uint32_t* __restrict__ ac, uint64_t& str) {
    int len = 0;
    str = 0ull;
    auto put = [&](uint32_t code, int n) {
        str |= (uint64_t)code << (64 - len - n);
        len += n;
    };
    if (v != 0) {
        const uint64_t below = nz & ((1ull << k) - 1ull);
        const int prev = below ? 63 - __clzll((long long)below) : 0;
        int run = k - prev - 1;
        const uint32_t zrl = ac[0xF0];
        while (run > 15) {
            put(zrl & 0xFFFFu, (int)(zrl >> 16));
            run -= 16;
        }
        const int m = cat_bits(v);
        const uint32_t e = ac[(run << 4) | m];
        put(e & 0xFFFFu, (int)(e >> 16));
        put(mag_bits(v, m), m);
    } else if (k == 63) {  // EOB after the last nonzero coefficient
        const uint32_t e = ac[0x00];
        put(e & 0xFFFFu, (int)(e >> 16));
    }
    return len;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// Exclusive scan of one value per thread over the workgroup; returns the total.
__device__ uint32_t wg_scan(uint32_t& v, uint32_t* lds_waves) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
    }
    if (lane == 63) lds_waves[w] = inc;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int k = 0; k < kJpegThreads / 64; ++k) {
        if (k < w) base += lds_waves[k];
        total += lds_waves[k];
    }
    v = base + inc - v;
    __syncthreads();
    return total;
}

// The forward transform of one block (fdct_block) + its AC bit count (acbits[block]).
__global__ __launch_bounds__(64) void k_jpeg_fdct_bits(const uchar4* __restrict__ rgba, int W, int H, int mcux,
                                                       const float* __restrict__ tab,
                                                       const uint32_t* __restrict__ huff,
                                                       int16_t* __restrict__ out, uint32_t* __restrict__ acbits) {
    __shared__ int q[64];
    const int blk = blockIdx.x % 6;
    const int t = threadIdx.x;
    const int v = fdct_block(rgba, W, H, mcux, tab, out, blk);
    q[t] = v;
    __syncthreads();
    const int z = q[c_zigzag[t]];
    const uint64_t nz = __ballot(z != 0 && t > 0);
    uint64_t str;
    const int len = t > 0 ? ac_lane(z, t, nz, huff + (blk < 4 ? 256 : 768), str) : 0;
    const uint32_t tot = wave_sum((uint32_t)len);
    if (t == 0) acbits[blockIdx.x] = tot;
}

__device__ __forceinline__ int dc_pred_block(int b) {  // previous block of b's component in its row, or -1
    const int k = b % 6;
    if (k >= 1 && k <= 3) return b - 1;
    if (b < 6) return -1;
    return b - (k == 0 ? 3 : 6);
}

// Block bit offsets within each row (DC bits added here), row totals, zeroed words.
__global__ __launch_bounds__(kJpegThreads) void k_jpeg_scan(const int16_t* __restrict__ coeffs, int mcux,
                                                            const uint32_t* __restrict__ huff,
                                                            const uint32_t* __restrict__ acbits,
                                                            uint32_t* __restrict__ blk_off,
                                                            uint32_t* __restrict__ row_bits,
                                                            uint32_t* __restrict__ ready,
                                                            uint32_t* __restrict__ scratch, size_t scratch_words) {
    __shared__ uint32_t ws[kJpegThreads / 64];
    const int my = blockIdx.x;
    const int nblk = mcux * 6;
    const int chunk = (nblk + kJpegThreads - 1) / kJpegThreads;
    const int b0 = min(nblk, (int)threadIdx.x * chunk), b1 = min(nblk, b0 + chunk);
    const size_t rb = (size_t)my * nblk;
    uint32_t sum = 0;
    for (int b = b0; b < b1; ++b) {
        const int p = dc_pred_block(b);
        const int diff = coeffs[(rb + b) * 64] - (p >= 0 ? coeffs[(rb + p) * 64] : 0);
        const int n = cat_bits(diff);
        const uint32_t e = huff[((b % 6) < 4 ? 0 : 512) + n];
        sum += (e >> 16) + n + acbits[rb + b];
    }
    uint32_t off = sum;
    const uint32_t total = wg_scan(off, ws);
    for (int b = b0; b < b1; ++b) {
        blk_off[rb + b] = off;
        const int p = dc_pred_block(b);
        const int diff = coeffs[(rb + b) * 64] - (p >= 0 ? coeffs[(rb + p) * 64] : 0);
        const int n = cat_bits(diff);
        const uint32_t e = huff[((b % 6) < 4 ? 0 : 512) + n];
        off += (e >> 16) + n + acbits[rb + b];
    }
    uint32_t* row = scratch + (size_t)my * scratch_words;
    const uint32_t nw = (total + 31u) / 32u;
    for (uint32_t w = threadIdx.x; w < nw; w += kJpegThreads) row[w] = 0u;
    if (threadIdx.x == 0) {
        row_bits[my] = total;
        ready[my] = 0u;
    }
}

// Bits [pos, pos + len) of a word array = the top len bits of str.
template <typename OrFn>
__device__ __forceinline__ void or_bits(uint32_t pos, uint64_t str, int len, OrFn&& orw) {
    if (len <= 0) return;
    const uint32_t w = pos >> 5;
    const int sh = (int)(pos & 31u);
    orw(w, (uint32_t)(str >> (32 + sh)));
    if (sh + len > 32) {
        const uint64_t rest = str << (32 - sh);
        orw(w + 1, (uint32_t)(rest >> 32));
        if (sh + len > 64) orw(w + 2, (uint32_t)rest);
    }
}

constexpr int kBlockWords = kJpegBlockMaxBytes / 4 + 2;  // a block's bits + alignment slack, in words

// One wave per block: the lanes' symbols are OR-ed into the block's words in
// LDS (aligned like the row: local bit = global bit - 32 * first word), then
// the wave writes them out: inner words stored, the first and last (shared
// with the neighbouring blocks) OR-ed atomically.
__global__ __launch_bounds__(kJpegThreads) void k_jpeg_emit(const int16_t* __restrict__ coeffs, int mcux, int nblocks,
                                                            const uint32_t* __restrict__ huff,
                                                            const uint32_t* __restrict__ blk_off,
                                                            const uint32_t* __restrict__ row_bits,
                                                            uint32_t* __restrict__ scratch, size_t scratch_words) {
    __shared__ uint32_t words[kJpegThreads / 64][kBlockWords];
    const int wv = threadIdx.x >> 6;
    const int gb = blockIdx.x * (kJpegThreads / 64) + wv;
    if (gb >= nblocks) return;
    const int t = threadIdx.x & 63;
    const int nblk = mcux * 6;
    const int my = gb / nblk, b = gb % nblk;
    uint32_t* lw = words[wv];
    for (int i = t; i < kBlockWords; i += 64) lw[i] = 0u;
    const int16_t* blk = coeffs + (size_t)gb * 64;
    const int z = blk[c_zigzag[t]];
    const uint64_t nz = __ballot(z != 0 && t > 0);
    const bool luma = (b % 6) < 4;
    uint64_t str = 0ull;
    int len;
    if (t == 0) {  // DC difference
        const int p = dc_pred_block(b);
        const int diff = z - (p >= 0 ? coeffs[(size_t)(gb - b + p) * 64] : 0);
        const int n = cat_bits(diff);
        const uint32_t e = huff[(luma ? 0 : 512) + n];
        const int cl = (int)(e >> 16);
        str = ((uint64_t)(e & 0xFFFFu) << (64 - cl)) | (n ? (uint64_t)mag_bits(diff, n) << (64 - cl - n) : 0ull);
        len = cl + n;
    } else {
        len = ac_lane(z, t, nz, huff + (luma ? 256 : 768), str);
    }
    uint32_t inc = (uint32_t)len;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off);
        if (t >= off) inc += o;
    }
    const uint32_t start = blk_off[gb];
    const uint32_t nbits = __shfl(inc, 63);
    const uint32_t w0 = start >> 5;
    __builtin_amdgcn_wave_barrier();
    or_bits((start & 31u) + inc - (uint32_t)len, str, len, [&](uint32_t w, uint32_t v) {
        if (v) atomicOr(&lw[w], v);
    });
    __builtin_amdgcn_wave_barrier();
    if (nbits == 0) return;
    const uint32_t nw = ((start & 31u) + nbits + 31u) >> 5;
    uint32_t* row = scratch + (size_t)my * scratch_words + w0;
    for (uint32_t i = t; i < nw; i += 64) {
        const uint32_t v = lw[i];
        if (i == 0 || i + 1 == nw) atomicOr(&row[i], v);
        else row[i] = v;
    }
    (void)row_bits;
}

// 1-bit padding of the row's last byte and byte stuffing, straight into the
// file stream in pinned host memory ([0, 8) length, [16, ...) bytes): each row
// publishes its stuffed length (ready[r] = len + 1, zeroed by k_jpeg_scan) as
// soon as it is counted, then sums the lengths of the rows before it (rows
// are dispatched in order and publish before waiting, so the wait ends), and
// writes its bytes + RSTn (EOI after the last row) at that offset.
__global__ __launch_bounds__(kJpegThreads) void k_jpeg_finish(const uint32_t* __restrict__ row_bits,
                                                              const uint32_t* __restrict__ scratch,
                                                              size_t scratch_words, uint32_t* __restrict__ ready,
                                                              int mcuy, uint8_t* __restrict__ host) {
    __shared__ uint32_t ws[kJpegThreads / 64];
    __shared__ uint32_t s_base;
    const int my = blockIdx.x;
    const uint32_t total = row_bits[my];
    const uint32_t* row = scratch + (size_t)my * scratch_words;
    const uint32_t nbytes = (total + 7u) >> 3;
    const uint32_t bchunk = (nbytes + kJpegThreads - 1) / kJpegThreads;
    const uint32_t j0 = min(nbytes, threadIdx.x * bchunk), j1 = min(nbytes, j0 + bchunk);
    const uint32_t pad = (8u - (total & 7u)) & 7u;
    auto byte_at = [&](uint32_t j) -> uint32_t {
        uint32_t v = (row[j >> 2] >> (24u - 8u * (j & 3u))) & 0xFFu;
        if (j + 1 == nbytes) v |= (1u << pad) - 1u;
        return v;
    };
    uint32_t nff = 0;
    for (uint32_t j = j0; j < j1; ++j) nff += byte_at(j) == 0xFFu ? 1u : 0u;
    const uint32_t total_ff = wg_scan(nff, ws);  // nff: 0xFF bytes before this thread's first byte
    const uint32_t len = nbytes + total_ff + 2u;  // + RSTn / EOI
    if (threadIdx.x == 0) {
        __hip_atomic_store(&ready[my], len + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        s_base = 0u;
    }
    __syncthreads();
    uint32_t part = 0;
    for (int q = threadIdx.x; q < my; q += kJpegThreads) {
        uint32_t v;
        while ((v = __hip_atomic_load(&ready[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
            __builtin_amdgcn_s_sleep(1);
        part += v - 1u;
    }
    part = wave_sum(part);
    if ((threadIdx.x & 63) == 0 && part) atomicAdd(&s_base, part);
    __syncthreads();
    uint8_t* out = host + 16 + s_base;
    uint32_t o = j0 + nff;
    for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t v = byte_at(j);
        out[o++] = (uint8_t)v;
        if (v == 0xFFu) out[o++] = 0;
    }
    if (threadIdx.x == 0) {
        out[len - 2] = 0xFF;
        out[len - 1] = my + 1 < mcuy ? (uint8_t)(0xD0 + (my & 7)) : (uint8_t)0xD9;
        if (my + 1 == mcuy) *reinterpret_cast<uint64_t*>(host) = (uint64_t)s_base + len;
    }
}

}  // namespace

size_t jpeg_row_scratch_words(int W) { return (size_t)((W + 15) / 16) * 6 * kJpegBlockMaxBytes / 4 + 2; }
static size_t jpeg_row_stuffed_bytes(int W) { return (size_t)((W + 15) / 16) * 6 * kJpegBlockMaxBytes * 2 + 16; }
size_t jpeg_stream_max_bytes(int W, int H) {
    return (size_t)((H + 15) / 16) * (jpeg_row_stuffed_bytes(W) + 2) + 16;
}

void jpeg_encode_device(const uint8_t* d_rgba, int W, int H, const float* d_tab, const uint32_t* d_huff,
                        int16_t* d_coeffs, JpegDevBufs& b, uint8_t* host_out, hipStream_t st) {
    const int mcux = (W + 15) / 16, mcuy = (H + 15) / 16;
    const int nblocks = mcux * mcuy * 6;
    const size_t sw = jpeg_row_scratch_words(W);
    k_jpeg_fdct_bits<<<nblocks, 64, 0, st>>>(reinterpret_cast<const uchar4*>(d_rgba), W, H, mcux, d_tab, d_huff,
                                             d_coeffs, b.acbits);
    k_jpeg_scan<<<mcuy, kJpegThreads, 0, st>>>(d_coeffs, mcux, d_huff, b.acbits, b.blk_off, b.row_bits, b.ready,
                                               b.scratch, sw);
    k_jpeg_emit<<<(nblocks + 3) / 4, kJpegThreads, 0, st>>>(d_coeffs, mcux, nblocks, d_huff, b.blk_off, b.row_bits,
                                                             b.scratch, sw);
    k_jpeg_finish<<<mcuy, kJpegThreads, 0, st>>>(b.row_bits, b.scratch, sw, b.ready, mcuy, host_out);
    RR_HIP(hipGetLastError());
}

}  // namespace rr
