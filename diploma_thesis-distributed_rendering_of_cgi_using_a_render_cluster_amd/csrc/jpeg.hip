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

// One 64-thread workgroup per 8x8 block; blocks 0..3 = Y (2x2), 4 = Cb, 5 = Cr.
// tab: dct[64] | qinv_luma[64] | qinv_chroma[64].
__global__ __launch_bounds__(64) void k_jpeg_fdct(const uchar4* __restrict__ rgba, int W, int H, int mcux,
                                                  const float* __restrict__ tab, int16_t* __restrict__ out) {
    __shared__ float in[64];
    __shared__ float tmp[64];
    const int blk = blockIdx.x % 6;
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
        out[((size_t)mcu * 6 + blk) * 64 + 8 * v + u] = (int16_t)rintf(s * qinv[8 * v + u]);
    }
}

}  // namespace

void jpeg_fdct_device(const uint8_t* d_rgba, int W, int H, const float* d_tab, int16_t* d_out, hipStream_t st) {
    const int mcux = (W + 15) / 16, mcuy = (H + 15) / 16;
    k_jpeg_fdct<<<mcux * mcuy * 6, 64, 0, st>>>(reinterpret_cast<const uchar4*>(d_rgba), W, H, mcux, d_tab, d_out);
    RR_HIP(hipGetLastError());
}

}  // namespace rr
