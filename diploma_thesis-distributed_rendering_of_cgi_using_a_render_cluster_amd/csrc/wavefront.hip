// Wavefront path tracer. Per chunk of spp_chunk samples x all
// pixels:
//   K-primary  (K6 raygen + K7 closest-hit traversal + K9 shade, bounce 0):
//              the camera path lives in registers; it writes its radiance
//              record and appends, through wave-level ballot/popcount queue
//              compaction (K8), only what continues: the next ray + throughput
//              to the dense path queue and the NEE ray to the shadow queue;
//   K-shadow   (K10 any-hit): one launch per bounce over the dense shadow
//              queue, adds the unoccluded NEE contribution to the radiance
//              record;
//   K-extend   (K7 + K9 + K8, bounce >= 1): one launch per bounce over the
//              dense path queue (coalesced SoA reads, compacted writes);
//   K-accumulate (K11 + K12 on the last chunk): film += chunk radiance in
//              sample order, then mean -> exposure -> view transform -> 8-bit.
// Every kernel is a persistent grid-stride loop over a device-side queue count,
// so a frame is one stream of launches with no host round trip.
//
// HBM per camera path: 16 B radiance write + 16 B accumulate read; per
// continuing path per bounce: 48 B state write + read, 32 B radiance RMW;
// per shadow ray: 48 B write + read (+32 B RMW). The arithmetic is the
// uncontracted, libm-free form of rr_device.h and matches oracle/rr_oracle.c
// bit for bit.
//
// Replaces the per-pixel, per-sample path integration of Cycles behind
// bpy.ops.render.render (/root/reference/scripts/render-timing-script.py:90).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device.hpp"

namespace rr {

namespace {

struct LightsMats {
    const float* lights;     // n_lights * RR_LIGHT_FLOATS
    const float* materials;  // RR_MAT_FLOATS each
    const float* filter;     // kFilterTableSize
    const float* srgb;       // kSrgbLutSize + 1
};

constexpr int kFilterN = 1024;
constexpr int kSrgbN = 4096;
constexpr int kLightF = 12;
constexpr int kMatF = 12;
constexpr float kFltMax = 3.402823466e+38f;

// Dense queue state (SoA, ping-pong per bounce).
struct PathQueue {
    float4* o;  // origin.xyz, path id (int bits)
    float4* d;  // direction.xyz, 0
    float4* t;  // throughput.xyz, 0
};
struct ShadowQueue {
    float4* o;  // origin.xyz, path id (int bits)
    float4* d;  // direction.xyz, tmax
    float4* c;  // contribution.xyz, 0
};

__device__ __forceinline__ Mat load_mat(const float* __restrict__ mats, int id) {
    const float* m = mats + kMatF * id;
    Mat r;
    r.base = mk3(m[0], m[1], m[2]);
    r.metallic = m[3];
    r.specular = m[4];
    r.roughness = m[5];
    r.ior = m[6];
    r.emission = mk3(m[7], m[8], m[9]);
    r.model = (int)m[10];
    return r;
}

// Camera ray for (pixel, sample): filter-importance-sampled subpixel position,
// pinhole through the sensor plane at unit distance, z-depth clipping.
__device__ __forceinline__ void camera_ray(const FrameConsts& fc, const float* __restrict__ filt, int pix,
                                           uint32_t key, float3& o, float3& d, float& tmin, float& tmax) {
    const int px = pix % fc.W;
    const int py = pix / fc.W;
    const float fx = (float)px + 0.5f + table_lerp(filt, kFilterN, rng(key, 0));
    const float fy = (float)py + 0.5f + table_lerp(filt, kFilterN, rng(key, 1));
    const float sx = (fx * fc.inv_w2 - 1.0f) * fc.half_w;
    const float sy = (1.0f - fy * fc.inv_h2) * fc.half_h;
    const float len = sqrtf(sx * sx + sy * sy + 1.0f);
    const float3 dw = mk3(fc.cam_right.x * sx + fc.cam_up.x * sy - fc.cam_back.x,
                          fc.cam_right.y * sx + fc.cam_up.y * sy - fc.cam_back.y,
                          fc.cam_right.z * sx + fc.cam_up.z * sy - fc.cam_back.z);
    const float il = 1.0f / len;
    d = scl3(dw, il);
    o = fc.cam_pos;
    tmin = fc.clip_start * len;
    tmax = fc.clip_end * len;
}

struct ShadeOut {
    bool cont, shadow;
    float3 o, d, T;          // continuation ray + throughput
    float3 so, sd, sc;       // shadow ray + pending contribution
    float sdist;
};

RR_D void add_to(float3& L, float3 c) {
    L.x = L.x + c.x;
    L.y = L.y + c.y;
    L.z = L.z + c.z;
}

// K9: shade one path at `bounce` given its closest hit; L updated in place.
__device__ __forceinline__ void shade(const FrameConsts& fc, int bounce, const LightsMats& lm,
                                      const TriPack* __restrict__ tris, float3 o, float3 d, float3 T,
                                      const Hit& h, uint32_t key, float3& L, ShadeOut& out) {
    out.cont = false;
    out.shadow = false;
    if (h.idx < 0) {
        float3 c = mul3(T, fc.world);
        if (bounce > 0) c = clamp_contrib(c, fc.clamp_indirect);
        add_to(L, c);
        return;
    }
    const TriPack tp = tris[h.idx];
    const float3 e1 = xyz(tp.p1), e2 = xyz(tp.p2);
    const Mat m = load_mat(lm.materials, f2i(tp.p1.w));
    const float t = h.t;
    const float3 P = mk3(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
    float3 N = norm3(cross3(e1, e2));
    if (dot3(N, d) > 0.0f) N = mk3(-N.x, -N.y, -N.z);
    const float3 wo = mk3(-d.x, -d.y, -d.z);
    if (m.emission.x != 0.0f || m.emission.y != 0.0f || m.emission.z != 0.0f) {
        float3 c = mul3(T, m.emission);
        if (bounce > 0) c = clamp_contrib(c, fc.clamp_indirect);
        add_to(L, c);
    }
    if (bounce >= fc.max_bounces) return;
    const uint32_t dim0 = 2u + (uint32_t)(kDimsPerBounce * bounce);
    const float3 Po = offset_ray(P, N);
    // next-event estimation toward one uniformly chosen light
    if (fc.n_lights > 0) {
        int li = (int)(rng(key, dim0) * (float)fc.n_lights);
        if (li > fc.n_lights - 1) li = fc.n_lights - 1;
        const float* lt = lm.lights + kLightF * li;
        float3 wi, Li;  // Li: radiance x cos_light / pdf (solid angle), i.e. I*cos/d^2
        float dist;
        if (lt[0] == 0.0f) {  // point / disk light
            const float3 lp = mk3(lt[1], lt[2], lt[3]);
            const float radius = lt[7];
            const float3 I = mk3(lt[8], lt[9], lt[10]);
            const float3 tl = sub3(lp, P);
            const float dl2 = dot3(tl, tl);
            if (radius > 0.0f) {
                const float3 wl = scl3(tl, 1.0f / sqrtf(dl2));
                float3 b1, b2;
                make_onb(wl, b1, b2);
                float dx, dy;
                concentric_disk(rng(key, dim0 + 1u), rng(key, dim0 + 2u), dx, dy);
                dx = dx * radius;
                dy = dy * radius;
                const float3 sp = mk3(lp.x + b1.x * dx + b2.x * dy, lp.y + b1.y * dx + b2.y * dy,
                                      lp.z + b1.z * dx + b2.z * dy);
                const float3 ts = sub3(sp, P);
                const float ds2 = dot3(ts, ts);
                dist = sqrtf(ds2);
                wi = scl3(ts, 1.0f / dist);
                const float cl = fabsf(dot3(wl, wi));
                Li = scl3(I, cl / ds2);
            } else {
                dist = sqrtf(dl2);
                wi = scl3(tl, 1.0f / dist);
                Li = scl3(I, 1.0f / dl2);
            }
        } else {  // sun: delta direction, irradiance
            wi = mk3(-lt[4], -lt[5], -lt[6]);
            dist = kFltMax;
            Li = mk3(lt[8], lt[9], lt[10]);
        }
        const float cosN = dot3(N, wi);
        if (cosN > 0.0f) {
            float pdf;
            const float ps = spec_prob(m, dot3(N, wo));
            const float3 f = bsdf_eval(m, N, wo, wi, ps, pdf);
            const float k = cosN * (float)fc.n_lights;
            float3 c = mk3(T.x * f.x * k * Li.x, T.y * f.y * k * Li.y, T.z * f.z * k * Li.z);
            if (bounce > 0) c = clamp_contrib(c, fc.clamp_indirect);
            if (max3f(c) > 0.0f) {
                out.shadow = true;
                out.so = Po;
                out.sd = wi;
                out.sdist = dist;
                out.sc = c;
            }
        }
    }
    // continue the path
    float3 wi, f;
    float pdf;
    if (!bsdf_sample(m, N, wo, rng(key, dim0 + 3u), rng(key, dim0 + 4u), rng(key, dim0 + 5u), wi, f, pdf))
        return;
    const float cosL = dot3(N, wi);
    if (!(cosL > 0.0f)) return;
    const float k = cosL / pdf;
    T = mk3(T.x * f.x * k, T.y * f.y * k, T.z * f.z * k);
    if (!(max3f(T) > 0.0f)) return;
    if (bounce >= kRrStartBounce) {
        const float q = fminf(max3f(T), 1.0f);
        if (rng(key, dim0 + 6u) >= q) return;
        T = mk3(T.x / q, T.y / q, T.z / q);
    }
    out.cont = true;
    out.o = Po;
    out.d = wi;
    out.T = T;
}

// K8: wave-aggregated slot allocation (ballot + popcount, one atomic per wave).
// Every lane of the wave must call it.
__device__ __forceinline__ int wave_slot(bool want, int32_t* __restrict__ cnt) {
    const uint64_t mask = __ballot(want);
    if (mask == 0ull) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(cnt, __popcll(mask));
    base = __shfl(base, leader);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    return want ? base + __popcll(mask & lt) : -1;
}

__device__ __forceinline__ void emit(const ShadeOut& so, int pid, PathQueue out, int32_t* cnt_out,
                                     ShadowQueue sq, int32_t* cnt_sh) {
    const int s1 = wave_slot(so.cont, cnt_out);
    if (s1 >= 0) {
        out.o[s1] = make_float4(so.o.x, so.o.y, so.o.z, i2f(pid));
        out.d[s1] = make_float4(so.d.x, so.d.y, so.d.z, 0.0f);
        out.t[s1] = make_float4(so.T.x, so.T.y, so.T.z, 0.0f);
    }
    const int s2 = wave_slot(so.shadow, cnt_sh);
    if (s2 >= 0) {
        sq.o[s2] = make_float4(so.so.x, so.so.y, so.so.z, i2f(pid));
        sq.d[s2] = make_float4(so.sd.x, so.sd.y, so.sd.z, so.sdist);
        sq.c[s2] = make_float4(so.sc.x, so.sc.y, so.sc.z, 0.0f);
    }
}

// Traversal-count reduction (RR_FLAG_COUNT_TRAVERSAL only).
__device__ __forceinline__ void flush_counts(unsigned long long* __restrict__ tc, int slot, uint32_t nv,
                                             uint32_t nt) {
    unsigned long long a = nv, b = nt;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&tc[slot], a);
        atomicAdd(&tc[slot + 1], b);
    }
}

// K-primary: raygen + closest hit + shade of bounce 0 for every camera path.
template <bool kCount, int kMinWaves = 1>
__global__ __launch_bounds__(kBlock, kMinWaves) void k_primary(FrameConsts fc, LightsMats lm, const BvhNode* __restrict__ nodes,
                                                    const TriPack* __restrict__ tris, int np,
                                                    float4* __restrict__ rad, PathQueue out,
                                                    int32_t* __restrict__ cnt_out, ShadowQueue sq,
                                                    int32_t* __restrict__ cnt_sh, int32_t* __restrict__ spill,
                                                    unsigned long long* __restrict__ tc) {
    __shared__ int lds_stack[kLdsStack * kBlock];
    const int lane = threadIdx.x & 63;
    const int gtid = blockIdx.x * kBlock + threadIdx.x;
    const int stride = gridDim.x * kBlock;
    TravStack st{lds_slot(&lds_stack[threadIdx.x]), spill + gtid, stride, 0};
    TravCount cnt;
    for (int i0 = gtid - lane; i0 < np; i0 += stride) {
        const int p = i0 + lane;
        ShadeOut so;
        so.cont = so.shadow = false;
        if (p < np) {
            const int sl = p / fc.npix;
            const int pix = p - sl * fc.npix;
            const uint32_t key = path_key(fc.seed, (uint32_t)pix, (uint32_t)(fc.first_sample + sl));
            float3 o, d;
            float tmin, tmax;
            camera_ray(fc, lm.filter, pix, key, o, d, tmin, tmax);
            Hit h;
            traverse<false, kCount>(nodes, tris, fc.n_tris, o, d, tmin, tmax, st, h, cnt);
            float3 L = mk3(0.0f, 0.0f, 0.0f);
            shade(fc, 0, lm, tris, o, d, mk3(1.0f, 1.0f, 1.0f), h, key, L, so);
            rad[p] = make_float4(L.x, L.y, L.z, 0.0f);
        }
        emit(so, p, out, cnt_out, sq, cnt_sh);
    }
    if (kCount) flush_counts(tc, 0, cnt.nodes, cnt.tris);
}

// K-extend: closest hit + shade of bounce b >= 1 over the dense path queue.
template <bool kCount>
__global__ __launch_bounds__(kBlock) void k_extend(FrameConsts fc, int bounce, LightsMats lm,
                                                   const BvhNode* __restrict__ nodes,
                                                   const TriPack* __restrict__ tris,
                                                   const int32_t* __restrict__ cnt_in, PathQueue in,
                                                   float4* __restrict__ rad, PathQueue out,
                                                   int32_t* __restrict__ cnt_out, ShadowQueue sq,
                                                   int32_t* __restrict__ cnt_sh, int32_t* __restrict__ spill,
                                                   unsigned long long* __restrict__ tc) {
    __shared__ int lds_stack[kLdsStack * kBlock];
    const int count = *cnt_in;
    const int lane = threadIdx.x & 63;
    const int gtid = blockIdx.x * kBlock + threadIdx.x;
    const int stride = gridDim.x * kBlock;
    TravStack st{lds_slot(&lds_stack[threadIdx.x]), spill + gtid, stride, 0};
    TravCount cnt;
    int pid = 0;
    for (int i0 = gtid - lane; i0 < count; i0 += stride) {
        const int i = i0 + lane;
        ShadeOut so;
        so.cont = so.shadow = false;
        if (i < count) {
            const float4 a = in.o[i], b = in.d[i], c = in.t[i];
            pid = f2i(a.w);
            const float3 o = xyz(a), d = xyz(b);
            Hit h;
            traverse<false, kCount>(nodes, tris, fc.n_tris, o, d, 0.0f, kFltMax, st, h, cnt);
            const int sl = pid / fc.npix;
            const int pix = pid - sl * fc.npix;
            const uint32_t key = path_key(fc.seed, (uint32_t)pix, (uint32_t)(fc.first_sample + sl));
            const float4 L4 = rad[pid];
            float3 L = xyz(L4);
            shade(fc, bounce, lm, tris, o, d, xyz(c), h, key, L, so);
            rad[pid] = make_float4(L.x, L.y, L.z, 0.0f);
        }
        emit(so, pid, out, cnt_out, sq, cnt_sh);
    }
    if (kCount) flush_counts(tc, 2, cnt.nodes, cnt.tris);
}

// K10: shadow rays of one bounce; unoccluded -> radiance += contribution.
template <bool kCount>
__global__ __launch_bounds__(kBlock) void k_shadow(const BvhNode* __restrict__ nodes,
                                                   const TriPack* __restrict__ tris, int n_tris,
                                                   const int32_t* __restrict__ cnt_sh, ShadowQueue sq,
                                                   float4* __restrict__ rad, int32_t* __restrict__ spill,
                                                   unsigned long long* __restrict__ tc) {
    __shared__ int lds_stack[kLdsStack * kBlock];
    const int count = *cnt_sh;
    const int gtid = blockIdx.x * kBlock + threadIdx.x;
    const int stride = gridDim.x * kBlock;
    TravStack st{lds_slot(&lds_stack[threadIdx.x]), spill + gtid, stride, 0};
    TravCount cnt;
    for (int i = gtid; i < count; i += stride) {
        const float4 a = sq.o[i], b = sq.d[i];
        Hit h;
        if (!traverse<true, kCount>(nodes, tris, n_tris, xyz(a), xyz(b), 0.0f, b.w, st, h, cnt)) {
            const int pid = f2i(a.w);
            const float4 c = sq.c[i];
            float4 L = rad[pid];
            L.x = L.x + c.x;
            L.y = L.y + c.y;
            L.z = L.z + c.z;
            rad[pid] = L;
        }
    }
    if (kCount) flush_counts(tc, 4, cnt.nodes, cnt.tris);
}

// K11 (+K12 on the last chunk): film += radiance of this chunk's samples in
// sample order; then mean -> exposure -> view transform -> 8-bit.
__global__ __launch_bounds__(kBlock) void k_accumulate(FrameConsts fc, const float4* __restrict__ rad,
                                                       float4* __restrict__ film, int first_chunk,
                                                       int last_chunk, const float* __restrict__ srgb,
                                                       uchar4* __restrict__ out) {
    for (int pix = blockIdx.x * kBlock + threadIdx.x; pix < fc.npix; pix += gridDim.x * kBlock) {
        float4 acc = first_chunk ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : film[pix];
        for (int s = 0; s < fc.spp_chunk; ++s) {
            const float4 L = rad[(size_t)s * fc.npix + pix];
            acc.x = acc.x + L.x;
            acc.y = acc.y + L.y;
            acc.z = acc.z + L.z;
        }
        film[pix] = acc;
        if (last_chunk) {
            float c[3] = {acc.x * fc.inv_spp * fc.exposure_scale, acc.y * fc.inv_spp * fc.exposure_scale,
                          acc.z * fc.inv_spp * fc.exposure_scale};
            uint8_t q[3];
            for (int k = 0; k < 3; ++k) {
                float v = fminf(fmaxf(c[k], 0.0f), 1.0f);
                if (fc.view_transform == 0) v = srgb_oetf(v, srgb, kSrgbN);
                q[k] = quantize8(v);
            }
            out[pix] = make_uchar4(q[0], q[1], q[2], 255);
        }
    }
}

__global__ void k_debug_trace(const BvhNode* __restrict__ nodes, const TriPack* __restrict__ tris, int n_tris,
                              int n, const float4* __restrict__ rays, float4* __restrict__ hits,
                              int32_t* __restrict__ prims, uint8_t* __restrict__ occ,
                              int32_t* __restrict__ spill) {
    __shared__ int lds_stack[kLdsStack * kBlock];
    const int gtid = blockIdx.x * kBlock + threadIdx.x;
    const int nthreads = gridDim.x * kBlock;
    TravStack st{lds_slot(&lds_stack[threadIdx.x]), spill + gtid, nthreads, 0};
    TravCount cnt;
    for (int i = gtid; i < n; i += nthreads) {
        const float4 o = rays[2 * i], d = rays[2 * i + 1];
        Hit h;
        traverse<false>(nodes, tris, n_tris, xyz(o), xyz(d), o.w, d.w, st, h, cnt);
        hits[i] = make_float4(h.t, h.u, h.v, 0.0f);
        prims[i] = h.orig;
        Hit h2;
        occ[i] = traverse<true>(nodes, tris, n_tris, xyz(o), xyz(d), o.w, d.w, st, h2, cnt) ? 1 : 0;
    }
}

}  // namespace

int device_cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        RR_HIP(hipGetDevice(&dev));
        RR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (cus <= 0) cus = 256;
    }
    return cus;
}

int counters_per_chunk(int max_bounces) { return 2 * (max_bounces + 2); }

namespace {
// Persistent grid = resident blocks: CUs x blocks per CU the kernel's register
// and LDS budget admits (a grid-stride loop over more blocks than fit would
// only queue the surplus behind the first wave of blocks).
template <typename K>
int resident_grid(K kernel) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0)
        per_cu = 4;
    return device_cu_count() * per_cu;
}
struct Grids {
    int primary, primary5, extend, shadow, accum;
    Grids()
        : primary(resident_grid(k_primary<false>)), primary5(resident_grid(k_primary<false, 5>)),
          extend(resident_grid(k_extend<false>)),
          shadow(resident_grid(k_shadow<false>)),
          accum(resident_grid(k_accumulate)) {}
};
const Grids& grids() {
    static Grids g;
    return g;
}
inline int clamp_grid(long work, int resident) {
    const long g = (work + kBlock - 1) / kBlock;
    return (int)std::max<long>(1, std::min<long>(g, resident));
}
}  // namespace

void DevPaths::ensure_paths(size_t n) {
    if (grid_blocks == 0) grid_blocks = device_cu_count() * 8;
    if (n > cap) {
        for (DevBuf<float4>* b : {&rad, &ps_o[0], &ps_d[0], &ps_t[0], &ps_o[1], &ps_d[1], &ps_t[1], &sh_o, &sh_d,
                                  &sh_c})
            b->ensure(n);
        cap = n;
    }
    spill.ensure((size_t)kSpillStack * grid_blocks * kBlock);
}

void DevPaths::release() {
    for (DevBuf<float4>* b : {&rad, &ps_o[0], &ps_d[0], &ps_t[0], &ps_o[1], &ps_d[1], &ps_t[1], &sh_o, &sh_d,
                              &sh_c, &film})
        b->release();
    counters.release(); spill.release();
    rgba8.release(); filter_table.release(); srgb_lut.release(); lights.release(); materials.release();
    trav_counts.release();
    prof.release();
    cap = 0;
}

void render_frame_device(DevScene& s, DevPaths& p, const FrameConsts& base, int n_chunks, hipStream_t st) {
    const int npix = base.npix;
    const size_t npaths = (size_t)npix * base.spp_chunk;
    p.ensure_paths(npaths);
    p.film.ensure((size_t)npix);
    p.rgba8.ensure((size_t)npix * 4);
    const int cpc = counters_per_chunk(base.max_bounces);
    p.counters.ensure((size_t)cpc * n_chunks);
    RR_HIP(hipMemsetAsync(p.counters.ptr, 0, sizeof(int32_t) * cpc * n_chunks, st));
    LightsMats lm{p.lights.ptr, p.materials.ptr, p.filter_table.ptr, p.srgb_lut.ptr};
    unsigned long long* tc = nullptr;
    if (p.count_traversal) {
        p.trav_counts.ensure(6);
        RR_HIP(hipMemsetAsync(p.trav_counts.ptr, 0, 6 * sizeof(unsigned long long), st));
        tc = p.trav_counts.ptr;
    }
    PathQueue pq[2] = {{p.ps_o[0].ptr, p.ps_d[0].ptr, p.ps_t[0].ptr}, {p.ps_o[1].ptr, p.ps_d[1].ptr, p.ps_t[1].ptr}};
    ShadowQueue sq{p.sh_o.ptr, p.sh_d.ptr, p.sh_c.ptr};
    KernelProfiler& pr = p.prof;
    const Grids& G = grids();
    for (int c = 0; c < n_chunks; ++c) {
        FrameConsts fc = base;
        fc.first_sample = c * base.spp_chunk;
        fc.spp_chunk = base.spp_chunk;
        if (fc.first_sample + fc.spp_chunk > base.spp_total) fc.spp_chunk = base.spp_total - fc.first_sample;
        const int np = npix * fc.spp_chunk;
        int32_t* ext = p.counters.ptr + (size_t)cpc * c;  // ext[b]: paths entering bounce b (b >= 1)
        int32_t* shc = ext + (base.max_bounces + 2);      // shc[b]: shadow rays of bounce b
        pr.begin(st, RR_K_PRIMARY);
        // RR_TUNE_PRIMARY_WAVES=5: register-capped variant (A/B tuning knob)
        static const bool prim5 = getenv("RR_TUNE_PRIMARY_WAVES") && atoi(getenv("RR_TUNE_PRIMARY_WAVES")) == 5;
        auto kprim = tc ? k_primary<true> : (prim5 ? k_primary<false, 5> : k_primary<false>);
        kprim<<<clamp_grid(np, prim5 ? G.primary5 : G.primary), kBlock, 0, st>>>(fc, lm, s.nodes.ptr, s.tris.ptr, np, p.rad.ptr,
                                                                 pq[1], ext + 1, sq, shc, p.spill.ptr, tc);
        pr.end(st);
        for (int b = 0; b <= base.max_bounces; ++b) {
            if (b > 0) {
                pr.begin(st, RR_K_EXTEND);
                (tc ? k_extend<true> : k_extend<false>)<<<clamp_grid(np, G.extend), kBlock, 0, st>>>(fc, b, lm, s.nodes.ptr, s.tris.ptr, ext + b,
                                                                       pq[b & 1], p.rad.ptr, pq[(b + 1) & 1],
                                                                       ext + b + 1, sq, shc + b, p.spill.ptr, tc);
                pr.end(st);
            }
            pr.begin(st, RR_K_SHADOW);
            (tc ? k_shadow<true> : k_shadow<false>)<<<clamp_grid(np, G.shadow), kBlock, 0, st>>>(s.nodes.ptr, s.tris.ptr, s.n_tris, shc + b, sq,
                                                                   p.rad.ptr, p.spill.ptr, tc);
            pr.end(st);
        }
        const int ga = clamp_grid(npix, G.accum);
        pr.begin(st, RR_K_ACCUM);
        k_accumulate<<<ga, kBlock, 0, st>>>(fc, p.rad.ptr, p.film.ptr, c == 0 ? 1 : 0, c == n_chunks - 1 ? 1 : 0,
                                            p.srgb_lut.ptr, reinterpret_cast<uchar4*>(p.rgba8.ptr));
        pr.end(st);
    }
    RR_HIP(hipGetLastError());
}

void trace_batch_device(DevScene& s, DevPaths& p, int n, const float4* d_rays, float4* d_hits, int32_t* d_prims,
                        uint8_t* d_occ, hipStream_t st) {
    p.ensure_paths(1);
    const int g = (int)std::min<long>((n + kBlock - 1) / kBlock, p.grid_blocks);
    if (n > 0)
        k_debug_trace<<<g, kBlock, 0, st>>>(s.nodes.ptr, s.tris.ptr, s.n_tris, n, d_rays, d_hits, d_prims, d_occ,
                                            p.spill.ptr);
    RR_HIP(hipGetLastError());
}

}  // namespace rr
