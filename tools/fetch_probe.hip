// Calibration of the PMC byte counters for the traffic figures of the bench
// line (MI355X_MICROARCH.md: FETCH_SIZE x2 for streaming reads on gfx950).
// Two kernels with a known number of bytes read from HBM:
//   k_stream: every byte of a 1 GiB buffer once, coalesced dwordx4 loads;
//   k_gather: N random 64-byte nodes of a 4 GiB buffer (each a 64-B aligned
//             line, 4 dwordx4 loads by one lane, as the traversal kernels
//             fetch a QNode6), so almost every fetch misses L2 and MALL.
// Run under rocprofv3 --pmc FETCH_SIZE (and TCC_EA0_RDREQ_sum /
// TCC_EA0_RDREQ_64B_sum in a second pass); tools/fetch_probe.py divides the
// counters by the known bytes. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ in, size_t n4, float* __restrict__ out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.456f) out[0] = acc;  // keeps the loads; never true for the zeroed input
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// node k of thread i: a pseudo-random index below n_nodes
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ nodes, uint32_t n_nodes, int per_thread,
                                                float* __restrict__ out) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    float acc = 0.0f;
    uint32_t h = mix(t * 0x9E3779B9u + 1u);
    for (int k = 0; k < per_thread; ++k) {
        h = mix(h + (uint32_t)k);
        const float4* q = nodes + 4ull * (h % n_nodes);
        const float4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc += a.x + b.y + c.z + d.w;
    }
    if (acc == 123.456f) out[0] = acc;
}

int main(int argc, char** argv) {
    const size_t stream_bytes = (size_t)1 << 30;
    const size_t gather_bytes = (size_t)4 << 30;
    const uint32_t n_nodes = (uint32_t)(gather_bytes / 64);
    const int threads = 256 * 1024, per_thread = 16;  // 4M node fetches = 256 MiB
    float4 *bs, *bg;
    float* out;
    CHECK(hipMalloc(&bs, stream_bytes));
    CHECK(hipMalloc(&bg, gather_bytes));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(bs, 0, stream_bytes));
    CHECK(hipMemset(bg, 0, gather_bytes));
    for (int rep = 0; rep < 3; ++rep) {
        k_stream<<<2048, 256>>>(bs, stream_bytes / 16, out);
        k_gather<<<threads / 256, 256>>>(bg, n_nodes, per_thread, out);
    }
    CHECK(hipDeviceSynchronize());
    std::printf("{\"stream_bytes_per_launch\": %zu, \"gather_nodes_per_launch\": %d, \"gather_bytes_per_launch\": %zu}\n",
                stream_bytes, threads * per_thread, (size_t)threads * per_thread * 64);
    CHECK(hipFree(bs));
    CHECK(hipFree(bg));
    CHECK(hipFree(out));
    return 0;
}
