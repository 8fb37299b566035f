// Issue rate of v_fma_mix_f32 (fp16 operand widened inside the fma) against
// v_cvt_f32_ubyte0 + v_fma_f32 on gfx950 (research probe for the fp16-bound
// node experiment). Each lane runs kIters x 16 independent
// chains; the kernel time over the op count gives ops per clock per CU.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops \
//         -o tools/bin/mix_rate_probe tools/mix_rate_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 4096;
constexpr int kChains = 16;

// (each chain its own word, advanced every iteration, so no conversion is
// shared or hoisted; the integer add is the same in both kernels)
__global__ __launch_bounds__(256) void k_mix(const uint32_t* __restrict__ in, float* __restrict__ out, float s) {
    uint32_t w[kChains];
    float acc[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        acc[c] = (float)c;
        w[c] = in[threadIdx.x] + 0x00030003u * c;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            acc[c] = __builtin_fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)((c & 1) ? w[c] >> 16 : w[c])), s, acc[c]);
            w[c] += 0x00010001u;
        }
    }
    float r = 0.0f;
#pragma unroll
    for (int c = 0; c < kChains; ++c) r += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_cvt(const uint32_t* __restrict__ in, float* __restrict__ out, float s) {
    uint32_t w[kChains];
    float acc[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        acc[c] = (float)c;
        w[c] = in[threadIdx.x] + 0x03030303u * c;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            acc[c] = __builtin_fmaf((float)((w[c] >> (8 * (c & 3))) & 255u), s, acc[c]);
            w[c] += 0x01010101u;
        }
    }
    float r = 0.0f;
#pragma unroll
    for (int c = 0; c < kChains; ++c) r += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
    uint32_t* in;
    float* out;
    hipMalloc(&in, 256 * sizeof(uint32_t));
    hipMemset(in, 0, 256 * sizeof(uint32_t));
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 2; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (k == 0) k_mix<<<blocks, 256>>>(in, out, 1.0001f);
            else k_cvt<<<blocks, 256>>>(in, out, 1.0001f);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, a, b);
            const double fmas = (double)blocks * 256 * kIters * kChains;
            printf("%s rep %d: %.3f ms, %.1f G fma/s (%.2f lane-fmas per clock per CU at 2.4 GHz)\n",
                   k == 0 ? "fma_mix (fp16 operand)     " : "cvt_f32_ubyte + fma_f32    ", rep, ms, fmas / ms * 1e-6,
                   fmas / (ms * 1e-3) / 2.4e9 / cus);
        }
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
