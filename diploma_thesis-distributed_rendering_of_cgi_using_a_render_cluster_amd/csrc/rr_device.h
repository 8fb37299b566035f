// Device-side building blocks of the MI355X path tracer.
//
// Every floating-point expression here is written in the exact operation order
// of the CPU oracle (oracle/rr_oracle.c), compiled with contraction OFF on both
// sides (-ffp-contract=off plus the pragma below): a fused multiply-add appears
// only where the source spells fmaf() (v_fma_f32 here, the correctly rounded
// fmaf of C99 in the oracle, the same single rounding), IEEE division/sqrt
// (hipcc's default correctly rounded f32 div/sqrt), and no libm transcendentals on the
// per-sample path (sin/cos by the fixed polynomial of sincos_small, sRGB by a
// host-built table). That makes the GPU image reproducible bit for bit by the
// oracle (tests/test_gpu_parity.py).
//
// The reference has no renderer of its own: this replaces Blender Cycles'
// CPU path integration behind bpy.ops.render.render
// (/root/reference/scripts/render-timing-script.py:90).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RR_HD __host__ __device__ __forceinline__
#define RR_D __device__ __forceinline__

namespace rr {

// ---------------------------------------------------------------- layout ---
// BVH2 node, 64 B = one cache line. The two CHILD boxes live in the parent, so
// one node fetch decides both children (Karras LBVH, internal nodes 0..n-2).
//   f[0..2] left min   f[3..5] left max   f[6..8] right min  f[9..11] right max
//   i[12] left child   i[13] right child  (child < 0: leaf ~sorted_index)
struct alignas(16) BvhNode {
    float4 a, b, c;
    int4 d;
};
static_assert(sizeof(BvhNode) == 64, "node must be one 64-byte line");

// Quantised 6-wide node, the hierarchy of scenes traversed from HBM (split
// path): the PLOC BVH2 collapsed top down (each node's children
// start as its BVH2 root's two children and the largest internal one is opened
// until there are six), with the six child boxes stored as 8-bit offsets on a
// per-node grid: child lo/hi = org + q * 2^e per axis, q rounded outwards
// (exactly, in double, at build time), so each quantised box contains the
// child's box. Child references are implicit: the internal children of a node
// are consecutive nodes (breadth-first numbering) and its leaf children are
// consecutive triangles of the hierarchy's own triangle array (one triangle
// per leaf), both in slot order, so a node stores two bases and a mask and
// six children fit one 64-byte line (a 4-wide node with explicit links did
// too; six children per fetch take about a quarter fewer node visits per ray).
//   org.xyz  grid origin = the node box's lo corner
//   org.w    exponent bytes (ex + 128) | (ey + 128) << 8 | (ez + 128) << 16 | inner mask << 24
//   a        x: first internal child's node index, y: first leaf child's
//            triangle position, z / w: lo x / lo y of children 0..3 (byte c)
//   b        lo z, hi x, hi y, hi z of children 0..3 (byte c)
//   c        children 4, 5 as byte pairs: x (lo x, lo y), y (lo z, hi x), z (hi y, hi z),
//            w: mask of the used slots
// An unused slot has lo 255 and hi 0 on every axis, and its bit of c.w is 0:
// its box test always fails. oracle/rr_oracle.c q4_pack / trace4 restate the
// layout and the walk.
constexpr int kQWidth = 6;
struct alignas(16) QNode6 {
    float4 org;
    uint4 a, b, c;
};
static_assert(sizeof(QNode6) == 64, "quantised 6-wide node is 64 bytes");
RR_HD uint32_t q6_inner(const QNode6& n) { return (uint32_t)__builtin_bit_cast(int, n.org.w) >> 24; }
// child c's reference: >= 0 internal node, < 0 ~triangle position
RR_HD int q6_ref(const QNode6& n, int c) {
    const uint32_t inner = q6_inner(n), below = inner & ((1u << c) - 1u);
    return ((inner >> c) & 1u) ? (int)n.a.x + __builtin_popcount(below) : ~((int)n.a.y + (c - __builtin_popcount(below)));
}
RR_HD int q6_first_inner(const QNode6& n) { return (int)n.a.x; }
RR_HD int q6_first_leaf(const QNode6& n) { return (int)n.a.y; }

constexpr int kQExpMin = -64, kQExpMax = 100;

// Smallest e in [kQExpMin, kQExpMax] with 255 * 2^e >= ext (ext >= 0).
RR_HD int q4_exponent(double ext) {
    if (!(ext > 0.0)) return kQExpMin;
    int k;
    (void)frexp(ext, &k);  // ext = m 2^k, 0.5 <= m < 1: 255 * 2^(k-8) < 2^k, 255 * 2^(k-7) >= 2^k
    const int e = ldexp(255.0, k - 8) >= ext ? k - 8 : k - 7;
    return e < kQExpMin ? kQExpMin : (e > kQExpMax ? kQExpMax : e);
}
// Grid coordinate of a box bound, rounded down (lo) or up (hi), in [0, 255].
RR_HD uint32_t q4_quant(float v, float org, int e, bool up) {
    const double x = ((double)v - (double)org) * ldexp(1.0, -e);
    const double q = up ? ceil(x) : floor(x);
    return q <= 0.0 ? 0u : (q >= 255.0 ? 255u : (uint32_t)q);
}
// Reciprocal for the quantised slab test: finite for zero components (a ray
// parallel to an axis gets +-2^64, which keeps every plane distance finite).
RR_HD float q4_rcp(float x) { return fabsf(x) < 0x1p-64f ? (x < 0.0f ? -0x1p64f : 0x1p64f) : 1.0f / x; }
// Finite reciprocal of a ray direction for the slab tests (BVH2 and BVH4): one
// division for the three components when their product is at least 2^-100
// (then no component is below 2^-100 and nothing overflows), else q4_rcp per
// component. Traversal only decides which boxes are opened; the hits come from
// the triangle test, so the reciprocal's last bits never reach a pixel except
// through the oracle's identical walk.
RR_HD float3 rcp3(float3 d) {
    const float p = d.x * d.y;
    const float q = p * d.z;
    if (fabsf(q) >= 0x1p-100f) {
        const float r = 1.0f / q;
        return make_float3(r * (d.y * d.z), r * (d.x * d.z), r * p);
    }
    return make_float3(q4_rcp(d.x), q4_rcp(d.y), q4_rcp(d.z));
}

// Triangle in leaf order, 48 B: the three world vertices as the transform
// wrote them, with the original triangle id and material id in the .w lanes.
// The vertices themselves (not v0 and two edge vectors) so that triangles
// sharing a vertex see the same bits of it: the watertight test (woop_test)
// needs that. The edges e1 = v1 - v0, e2 = v2 - v0 of the shading normal are
// the same subtractions the build used to store (the same bits).
struct alignas(16) TriPack {
    float4 p0;  // v0.xyz, orig id (int bits)
    float4 p1;  // v1.xyz, material (int bits)
    float4 p2;  // v2.xyz, 0
};
static_assert(sizeof(TriPack) == 48, "tri pack is 48 bytes");
constexpr int kTriF4 = 3;  // float4s per TriPack (LDS staging)

// Leaf refs (< 0) name a range of sorted leaves: ~(first | (count - 1) << 28).
// The frame hierarchies use single-triangle leaves (count 1, ref = ~index):
// multi-triangle leaf ranges measured slower on every split-path config (one
// 02 frame at 16 spp / C5 at 8 spp: 1 -> 61.7 / 115.1 ms, 2 -> 70.0 / 132.5,
// 8 -> 121.7 / 229.9 ms); the range encoding stays for the BVH4 collapse.
RR_HD int leaf_ref(int first, int count) { return ~(first | ((count - 1) << 28)); }
RR_HD int leaf_first(int ref) { return (~ref) & 0x0FFFFFFF; }
RR_HD int leaf_count(int ref) { return ((~ref) >> 28) + 1; }

constexpr int kMaxLights = 64;
constexpr int kBlock = 256;         // threads per block for all path kernels
// Traversal stack per lane: kLdsStack entries in LDS, the rest (up to the
// oracle's ORC_MAXDEPTH = kStackCap = 80 in all) in a per-thread HBM spill
// area. 12 LDS entries (k_tiles, the debug walks; 16 with half the node copy
// measured 1-1.5 % slower on C5 in round 3, 256-thread blocks).
#ifndef RR_LDS_STACK
#define RR_LDS_STACK 12
#endif
constexpr int kStackCap = 80;
constexpr int kLdsStack = RR_LDS_STACK;
constexpr int kSpillStack = kStackCap - kLdsStack;
// The split path's trace kernels (round 6): 8 LDS entries per lane, 32 KB per
// 1,024-thread block, leave 48 KB for the top of the hierarchy (768 nodes,
// wavefront.hip kTopNodes) at two blocks per CU; against 12 entries and 512
// nodes: C5 frame slices -1.0 % (extension walks -1.8 %), 02 / 03 unchanged;
// 10 / 640 no better, 6 / 896 level, 4 / 1,024 +5 % (spills;
// profiles/r6_ab_lds_top.txt).
#ifndef RR_TRACE_LDS_STACK
#define RR_TRACE_LDS_STACK 8
#endif
constexpr int kTraceLdsStack = RR_TRACE_LDS_STACK;
// entries per lane of the spill area (DevPaths::spill): what the stack with
// the fewest LDS entries needs to reach kStackCap
constexpr int kSpillLane = kStackCap - (kTraceLdsStack < kLdsStack ? kTraceLdsStack : kLdsStack);
constexpr int kDimsPerBounce = 8;   // RNG dimensions consumed per bounce
constexpr int kRrStartBounce = 3;   // Russian roulette from this bounce on

// --------------------------------------------------------------- vectors ---
RR_HD float3 mk3(float x, float y, float z) { return make_float3(x, y, z); }
RR_HD float3 add3(float3 a, float3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
RR_HD float3 sub3(float3 a, float3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
RR_HD float3 mul3(float3 a, float3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
RR_HD float3 scl3(float3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
// Products of the vector helpers accumulate through fmaf (one rounding per
// multiply-add; dot: x first, then y, then z).
RR_HD float dot3(float3 a, float3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
RR_HD float3 cross3(float3 a, float3 b) {
    return mk3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
// a + b s, per component
RR_HD float3 madd3(float3 a, float3 b, float s) { return mk3(fmaf(b.x, s, a.x), fmaf(b.y, s, a.y), fmaf(b.z, s, a.z)); }
// x t + y u + z w (a point of the frame t, u, w)
RR_HD float3 frame3(float3 t, float3 u, float3 w, float x, float y, float z) {
    return mk3(fmaf(w.x, z, fmaf(u.x, y, t.x * x)), fmaf(w.y, z, fmaf(u.y, y, t.y * x)),
               fmaf(w.z, z, fmaf(u.z, y, t.z * x)));
}
RR_HD float3 norm3(float3 a) {
    const float inv = 1.0f / sqrtf(dot3(a, a));
    return scl3(a, inv);
}

// IEEE square root (the bits of sqrtf, which the oracle calls) for x = +-0 or
// x in [2^-96, FLT_MAX]. hipcc's correctly rounded sqrtf is v_sqrt_f32 (within
// 1 ulp) plus a correction that tries the neighbours s -+ 1 ulp by their
// residuals, wrapped in a 2^32 pre-scale for x < 2^-96 and a class test for
// zero / infinity; here the wrapping is left out (16 -> 9 instructions), which
// returns the same bits over that range: rr_debug_fastmath_check compares all
// 2^32 inputs with sqrtf on the device, 0 mismatches (tests/test_gpu_math.py). Every call site states
// why its argument is in range; sqrt_any handles the rest.
RR_HD float sqrt_rn(float x) {
#if __HIP_DEVICE_COMPILE__
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
    const float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
#else
    return sqrtf(x);
#endif
}
// Any x: sqrt_rn when every active lane's argument is in its range (one
// wave-uniform test), else the full sqrtf.
RR_HD float sqrt_any(float x) {
#if __HIP_DEVICE_COMPILE__
    if (__all((x >= 0x1p-96f && x <= 3.40282347e38f) || x == 0.0f)) return sqrt_rn(x);
#endif
    return sqrtf(x);
}
// IEEE reciprocal (the bits of 1.0f / b) for |b| in [2^-126, 2^126). hipcc's
// correctly rounded division is v_rcp_f32 refined by fused multiply-adds,
// between v_div_scale (which rescales operands near the exponent limits) and
// v_div_fixup (infinities, zeros, NaNs): 11 instructions. In that range
// neither wrapper changes anything, and the refinement alone (7 instructions)
// returns the same bits: rr_debug_fastmath_check compares every float with
// 1.0f / b on the device (tests/test_gpu_math.py).
RR_HD float rcp_rn(float b) {
#if __HIP_DEVICE_COMPILE__
    float r = __builtin_amdgcn_rcpf(b);
    r = fmaf(fmaf(-b, r, 1.0f), r, r);
    float q = fmaf(fmaf(-b, r, 1.0f), r, r);
    return fmaf(fmaf(-b, q, 1.0f), r, q);
#else
    return 1.0f / b;
#endif
}
// sqrt(x) and 1 / sqrt(x) (the bits of sqrtf and of 1.0f / sqrtf): sqrt_rn
// and rcp_rn when every active lane's x is in [2^-96, FLT_MAX] (the root then
// lies in [2^-48, 2^64], inside rcp_rn's range), else the IEEE operations.
RR_HD void sqrt_rcp_any(float x, float& s, float& r) {
#if __HIP_DEVICE_COMPILE__
    if (__all(x >= 0x1p-96f && x <= 3.40282347e38f)) {
        s = sqrt_rn(x);
        r = rcp_rn(s);
        return;
    }
#endif
    s = sqrtf(x);
    r = 1.0f / s;
}
// norm3 for |a|^2 in [2^-96, FLT_MAX] (sqrt_rn; same bits as norm3)
RR_HD float3 norm3_rn(float3 a) { return scl3(a, rcp_rn(sqrt_rn(dot3(a, a)))); }
RR_HD float3 norm3_any(float3 a) {
    float s, r;
    sqrt_rcp_any(dot3(a, a), s, r);
    return scl3(a, r);
}
RR_HD float max3f(float3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
RR_HD float3 xyz(float4 v) { return mk3(v.x, v.y, v.z); }

RR_HD int f2i(float f) { return __builtin_bit_cast(int, f); }
RR_HD float i2f(int i) { return __builtin_bit_cast(float, i); }

// Division by a runtime-constant divisor d >= 1 for 0 <= n < 2^31 with one
// mul_hi + shift (Granlund-Montgomery): k = 31 + ceil(log2 d), m = ceil(2^k / d)
// < 2^32; n*m/2^k = n/d + n*e/(d*2^k) with e = m*d - 2^k < d, and n*e < n*d <=
// 2^k keeps the floor exact. Integer results, so bit-exactness is unaffected.
struct FastDiv {
    uint32_t m;
    int sh;    // k - 32
    int one;   // d == 1
    static FastDiv make(uint32_t d) {
        FastDiv f{0u, 0, d == 1u ? 1 : 0};
        if (d <= 1u) return f;
        int c = 0;
        while ((1ull << c) < d) ++c;
        const int k = 31 + c;
        f.m = (uint32_t)(((1ull << k) + d - 1) / d);
        f.sh = k - 32;
        return f;
    }
    RR_D uint32_t div(uint32_t n) const { return one ? n : (__umulhi(n, m) >> sh); }
};

// ------------------------------------------------------------------- RNG ---
// Counter-based: u(dim) = hash(key + (dim+1)*golden), key = f(seed, pixel, sample).
// Independent of execution order, so wavefront (GPU) and scalar (oracle)
// traversals of the same path draw identical numbers.
RR_HD uint32_t hash_u32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// path_key = sample_key(pixel_key(seed, pixel), sample); the split lets a
// per-pixel sample loop hash the pixel once.
RR_HD uint32_t pixel_key(uint32_t seed, uint32_t pixel) { return hash_u32(hash_u32(seed) + pixel); }
RR_HD uint32_t sample_key(uint32_t pk, uint32_t sample) { return hash_u32(pk ^ (sample * 0x9E3779B9u + 0x7F4A7C15u)); }
RR_HD uint32_t path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return sample_key(pixel_key(seed, pixel), sample);
}
RR_HD float rng(uint32_t key, uint32_t dim) {
    return (float)(hash_u32(key + (dim + 1u) * 0x9E3779B9u) >> 8) * 5.9604644775390625e-08f;
}
// Two uniforms in [0, 1) from one hash, 16 bits each: the dimension pairs of
// a sample (camera subpixel; light pick + lobe choice; disk point; BSDF
// direction), half the hashes of one draw per dimension (each hash is two
// v_mul_lo_u32, quarter rate: a timing build with one multiply per hash was
// 2.3 % faster on 04vs). 2^-16 steps are far below the filter table's and the
// samplers' resolution.
RR_HD void rng2(uint32_t key, uint32_t dim, float& a, float& b) {
    const uint32_t h = hash_u32(key + (dim + 1u) * 0x9E3779B9u);
    a = (float)(h >> 16) * 1.52587890625e-05f;
    b = (float)(h & 0xffffu) * 1.52587890625e-05f;
}

// ------------------------------------------------------------- sampling ---
// sin/cos on |x| <= pi/4 (Cephes sinf/cosf kernels), fixed op order.
RR_HD void sincos_small(float x, float& s, float& c) {
    const float z = x * x;
    const float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    s = fmaf(ps * z, x, x);
    const float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    c = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
}

// Shirley-Chiu concentric square->disk map; angles stay in [-pi/4, pi/4].
// Written with selects instead of branches: each lane runs the operations of
// its own case (|a| > |b|: angle (pi/4) b/a, x = a cos, y = a sin; else angle
// (pi/4) a/b, x = b sin, y = b cos; a = b = 0: the origin), but a wave whose
// lanes fall in both cases pays for one division and one sincos, not two.
RR_HD void concentric_disk(float u1, float u2, float& x, float& y) {
    const float a = fmaf(2.0f, u1, -1.0f);
    const float b = fmaf(2.0f, u2, -1.0f);
    const bool wide = fabsf(a) > fabsf(b);
    const float num = wide ? b : a, r = wide ? a : b;
    float s, c;
    sincos_small(0.785398163397448f * (num / r), s, c);
    const bool origin = a == 0.0f && b == 0.0f;
    x = origin ? 0.0f : r * (wide ? c : s);
    y = origin ? 0.0f : r * (wide ? s : c);
}

// Orthonormal basis (Duff et al. 2017, branchless).
RR_HD void make_onb(float3 n, float3& b1, float3& b2) {
    const float sign = copysignf(1.0f, n.z);
    const float a = -rcp_rn(sign + n.z);  // |sign + n.z| in [1, 2] for a unit n; -1/x == -(1/x)
    const float b = n.x * n.y * a;
    b1 = mk3(fmaf(sign * n.x * n.x, a, 1.0f), sign * b, -sign * n.x);
    b2 = mk3(b, fmaf(n.y * n.y, a, sign), -n.y);
}

// Self-intersection-safe ray origin (Waechter & Binder, Ray Tracing Gems ch. 6).
RR_HD float offset_axis(float p, float n) {
    const int of = (int)(256.0f * n);
    const float pi = i2f(f2i(p) + ((p < 0.0f) ? -of : of));
    return fabsf(p) < 0.03125f ? fmaf(1.52587890625e-05f, n, p) : pi;
}
RR_HD float3 offset_ray(float3 p, float3 n) {
    return mk3(offset_axis(p.x, n.x), offset_axis(p.y, n.y), offset_axis(p.z, n.z));
}

// Piecewise-linear table read, u in [0,1] (t: global or LDS pointer).
template <typename FloatP>
RR_HD float table_lerp(FloatP t, int n, float u) {
    const float f = u * (float)(n - 1);
    int i = (int)f;
    if (i >= n - 1) return t[n - 1];
    if (i < 0) i = 0;
    const float fr = f - (float)i;
    return fmaf(t[i + 1] - t[i], fr, t[i]);
}
// The same read without the two range branches (each a divergent branch with
// its exec-mask bookkeeping on the per-sample path), for u in [0, 1] and a
// table whose entry t[n] repeats t[n - 1] (or u < 1): then i lies in
// [0, n - 1], and at i = n - 1 (u = 1) the lerp returns fmaf(0, 0, t[n - 1])
// = t[n - 1], the bits table_lerp returns.
template <typename FloatP>
RR_HD float table_lerp_padded(FloatP t, int n, float u) {
    const float f = u * (float)(n - 1);
    const int i = (int)f;
    const float fr = f - (float)i;
    return fmaf(t[i + 1] - t[i], fr, t[i]);
}

// ------------------------------------------------------- screen culling ---
// Screen-space bounds of the scene box [lo, hi] for the pinhole camera of
// wavefront.hip camera_ray (pos, right, up, back, half_w, half_h; image W x H):
// the 8 corners projected to subpixel coordinates (fx, fy of camera_ray), the
// bounding rectangle widened by one pixel. A camera ray whose (fx, fy) lies
// outside cannot meet the box, so it is a miss without traversal (every
// triangle lies in the box, and a hit point projects into the corners' convex
// hull; the pixel of slack covers rounding). Returns false — no culling — if a
// corner is not at least 1e-4 in front of the camera. oracle/rr_oracle.c
// screen_rect() is the same float computation.
RR_HD bool screen_rect(float3 pos, float3 right, float3 up, float3 back, float half_w, float half_h, float W,
                       float H, const float lo[3], const float hi[3], float rect[4]) {
    float x0 = 3.402823466e+38f, x1 = -3.402823466e+38f, y0 = 3.402823466e+38f, y1 = -3.402823466e+38f;
    for (int k = 0; k < 8; ++k) {
        const float3 v = mk3(((k & 1) ? hi[0] : lo[0]) - pos.x, ((k & 2) ? hi[1] : lo[1]) - pos.y,
                             ((k & 4) ? hi[2] : lo[2]) - pos.z);
        const float depth = -dot3(v, back);
        if (!(depth > 1.0e-4f)) return false;
        const float sx = dot3(v, right) / depth;
        const float sy = dot3(v, up) / depth;
        const float fx = (sx / half_w + 1.0f) * (W * 0.5f);
        const float fy = (1.0f - sy / half_h) * (H * 0.5f);
        x0 = fminf(x0, fx);
        x1 = fmaxf(x1, fx);
        y0 = fminf(y0, fy);
        y1 = fmaxf(y1, fy);
    }
    rect[0] = x0 - 1.0f;
    rect[1] = x1 + 1.0f;
    rect[2] = y0 - 1.0f;
    rect[3] = y1 + 1.0f;
    return true;
}

// ---------------------------------------------------------- intersection ---
// Watertight traversal. The triangle test (woop_test) decides a hit exactly in
// a 2D projection of the ray's own, so a ray never slips through the shared
// edge or vertex of two triangles; the box tests must then open every box that
// holds a triangle the test accepts. Their plane distances are rounded, so each
// test widens the box by a margin that covers the rounding of both tests:
// 2^-19 (32 units in the last place) of the larger of the coordinates involved
// (the box's distance from the ray origin plus its extent, per axis; the
// triangle test's projected vertices are exact to about 8 ulp of their distance
// from the origin, the plane distances to about 13). The margin is a distance
// along an axis; in t it is margin * |1/d| on that axis, subtracted from the
// near planes and added to the far ones. oracle/rr_oracle.c restates both.
constexpr float kBoxMargin = 0x1p-19f;

// Slab test against [bmin,bmax]; inclusive so equal-t candidates survive (the
// closest hit is then independent of traversal order, see closest_tri()).
// Plane distances t = fmaf(b, invd, oi) with oi = -(o invd) per ray (rcp3),
// each axis widened by its margin em (slab_margin).
RR_HD bool slab(float3 oi, float3 invd, float3 em, float bx0, float by0, float bz0, float bx1, float by1,
                float bz1, float tmin, float tmax, float& tnear) {
    const float tx0 = fmaf(bx0, invd.x, oi.x), tx1 = fmaf(bx1, invd.x, oi.x);
    const float ty0 = fmaf(by0, invd.y, oi.y), ty1 = fmaf(by1, invd.y, oi.y);
    const float tz0 = fmaf(bz0, invd.z, oi.z), tz1 = fmaf(bz1, invd.z, oi.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1) - em.x, fminf(ty0, ty1) - em.y), fmaxf(fminf(tz0, tz1) - em.z, tmin));
    const float tf = fminf(fminf(fmaxf(tx0, tx1) + em.x, fmaxf(ty0, ty1) + em.y), fminf(fmaxf(tz0, tz1) + em.z, tmax));
    tnear = tn;
    return tn <= tf;
}
// The BVH2 walk's margins in t for one ray: kBoxMargin * (|o|_inf + r) * |1/d|
// per axis, r = the largest |coordinate| of the scene box (every node box and
// vertex lies within it, so |b - o| <= |o|_inf + r bounds the rounding of every
// plane distance and projected vertex of the walk).
RR_HD float3 slab_margin(float3 o, float3 invd, float r) {
    const float m = (fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) + r) * kBoxMargin;
    return mk3(m * fabsf(invd.x), m * fabsf(invd.y), m * fabsf(invd.z));
}

// Watertight ray/triangle test (Woop, Benthin & Wald, JCGT 2(1) 2013). Per ray
// (make_shear): kz = the axis of the largest |d| component, kx, ky the next two
// cyclically, sx = d[kx] / d[kz], sy = d[ky] / d[kz], sz = 1 / d[kz]. Per
// triangle: the vertices relative to the origin, permuted to (kx, ky, kz)
// (rot3), sheared to 2D: x = a[kx] - sx a[kz], y = a[ky] - sy a[kz] — the
// projection along d, the same bits of a vertex for every triangle that shares
// it. The 2D edge functions U = cx by - cy bx, V = ax cy - ay cx, W = bx ay - by ax
// (no fused multiply-add, so an edge shared by two triangles gives exactly
// opposite values) decide the hit: inside iff U, V, W have no two opposite
// signs. One that rounds to 0 is recomputed exactly (edge_exact: the paper's
// double-precision fallback, done with two fused multiply-adds). So the projected
// triangles of a closed mesh cover the plane with no gap: a ray that meets the
// mesh hits at least one of its triangles, also on an edge or a vertex. Then
// det = U + V + W, t = (U az + V bz + W cz) sz / det (the kz coordinates scaled
// by sz), u = V / det and v = W / det (the weights of v1 and v2); the division
// only for rays that pass.
struct Shear {
    float sx, sy, sz;
    int kz;
};
// 1 / x: rcp_rn when every active lane's |x| is in [2^-126, 2^126) (one
// wave-uniform test), else the IEEE division.
RR_HD float rcp_any(float x) {
#if __HIP_DEVICE_COMPILE__
    if (__all(fabsf(x) >= 0x1p-126f && fabsf(x) < 0x1p126f)) return rcp_rn(x);
#endif
    return 1.0f / x;
}
// (a[kx], a[ky], a[kz]) for (kx, ky, kz) = (kz + 1, kz + 2, kz) mod 3.
RR_HD float3 rot3(float3 a, int kz) {
    const bool k0 = kz == 0, k1 = kz == 1;
    return mk3(k0 ? a.y : (k1 ? a.z : a.x), k0 ? a.z : (k1 ? a.x : a.y), k0 ? a.x : (k1 ? a.y : a.z));
}
RR_HD Shear make_shear(float3 d) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    Shear s;
    s.kz = ax >= ay ? (ax >= az ? 0 : 2) : (ay >= az ? 1 : 2);
    const float3 r = rot3(d, s.kz);
    s.sz = rcp_any(r.z);
    s.sx = r.x * s.sz;
    s.sy = r.y * s.sz;
    return s;
}
// An edge function a b - c d that rounded to 0 (e = 0): then the products
// p = a b and q = c d are equal floats, the exact value is the difference of
// their rounding errors fma(a, b, -p) - fma(c, d, -q) (each exact without
// underflow, and their difference is 0 only when the exact value is), which is
// also what the same difference in double rounds to; the swapped edge
// c d - a b of the neighbouring triangle gets exactly its negation. Other
// values pass through.
RR_HD float edge_exact(float a, float b, float c, float d, float e) {
    if (e != 0.0f) return e;
    return fmaf(a, b, -(a * b)) - fmaf(c, d, -(c * d));
}
// make_shear for a unit direction (camera rays): its largest component is at
// least 1/sqrt(3) in magnitude, inside rcp_rn's range, so no range test.
RR_HD int shear_axis(float3 d) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    return ax >= ay ? (ax >= az ? 0 : 2) : (ay >= az ? 1 : 2);
}
RR_HD Shear make_shear_unit(float3 d) {
    Shear s;
    s.kz = shear_axis(d);
    const float3 r = rot3(d, s.kz);
    s.sz = rcp_rn(r.z);
    s.sx = r.x * s.sz;
    s.sy = r.y * s.sz;
    return s;
}
// The test from the vertices relative to the origin, already permuted (a, b, c
// = rot3(v - o, kz)).
RR_HD bool woop_core(const Shear& s, float3 a, float3 b, float3 c, float& t, float& u, float& v) {
    const float ax = fmaf(-s.sx, a.z, a.x), ay = fmaf(-s.sy, a.z, a.y);
    const float bx = fmaf(-s.sx, b.z, b.x), by = fmaf(-s.sy, b.z, b.y);
    const float cx = fmaf(-s.sx, c.z, c.x), cy = fmaf(-s.sy, c.z, c.y);
    float U = cx * by - cy * bx;
    float V = ax * cy - ay * cx;
    float W = bx * ay - by * ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        U = edge_exact(cx, by, cy, bx, U);
        V = edge_exact(ax, cy, ay, cx, V);
        W = edge_exact(bx, ay, by, ax, W);
    }
    // the sign test (no two of U, V, W of opposite signs: min < 0 < max
    // rejects; fminf / fmaxf skip NaN as the comparisons do) and det != 0 as
    // one predicate: one divergent branch per test, not three
    const float det = U + V + W;
    const float mn = fminf(fminf(U, V), W), mx = fmaxf(fmaxf(U, V), W);
    if (((mn < 0.0f) & (mx > 0.0f)) | (det == 0.0f)) return false;
    const float T = fmaf(W, s.sz * c.z, fmaf(V, s.sz * b.z, U * (s.sz * a.z)));
    const float inv = 1.0f / det;
    t = T * inv;
    u = V * inv;
    v = W * inv;
    return true;
}
RR_HD bool woop_test(const Shear& s, float3 o, float3 v0, float3 v1, float3 v2, float& t, float& u, float& v) {
    return woop_core(s, rot3(sub3(v0, o), s.kz), rot3(sub3(v1, o), s.kz), rot3(sub3(v2, o), s.kz), t, u, v);
}

struct Hit {
    float t, u, v;
    int idx;   // leaf (sorted) index, -1 miss
    int orig;  // original triangle id, -1 miss
};

// Accept rule making the closest hit order-independent: smaller t wins; equal t
// -> smaller original id wins (bitwise on the predicates: one branch).
RR_HD bool closer(float t, int orig, float tmin, const Hit& h) {
    return (t > tmin) & ((t < h.t) | ((t == h.t) & (orig < h.orig)));
}
RR_HD void closest_tri(const TriPack& tp, int idx, const Shear& s, float3 o, float tmin, Hit& h) {
    float t, u, v;
    if (!woop_test(s, o, xyz(tp.p0), xyz(tp.p1), xyz(tp.p2), t, u, v)) return;
    const int orig = f2i(tp.p0.w);
    if (closer(t, orig, tmin, h)) {
        h.t = t;
        h.u = u;
        h.v = v;
        h.idx = idx;
        h.orig = orig;
    }
}

RR_HD void leaf_test(const TriPack& tp, int idx, const Shear& s, float3 o, float tmin, Hit& h) {
    closest_tri(tp, idx, s, o, tmin, h);
}


// Traversal stack: kLdsStack entries in LDS ([entry][thread] -> conflict-free
// ds_read_b32 across a wave), deeper entries in a per-thread HBM spill area.
// The LDS pointer carries its address space explicitly so push/pop compile to
// ds_write/ds_read (a generic pointer would become flat_* accesses).
typedef __attribute__((address_space(3))) int lds_int;
typedef __attribute__((address_space(3))) uint32_t lds_uint;
// LDS-staged scene data (wavefront.hip stage_scene): HIP's float4 has no
// address-space-3 copy, so 16-byte moves use a clang vector type.
typedef float rr_f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) rr_f4v lds_f4w;
typedef __attribute__((address_space(3))) const BvhNode lds_node;
typedef __attribute__((address_space(3))) const TriPack lds_tri;
typedef __attribute__((address_space(3))) const float lds_float;
RR_D float4 lds_ld4(const __attribute__((address_space(3))) rr_f4v* p) {
    const rr_f4v v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}
RR_D BvhNode load_node(const BvhNode* __restrict__ p, int i) { return p[i]; }
RR_D BvhNode load_node(lds_node* p, int i) {
    const __attribute__((address_space(3))) rr_f4v* q = (const __attribute__((address_space(3))) rr_f4v*)(p + i);
    BvhNode n;
    n.a = lds_ld4(q);
    n.b = lds_ld4(q + 1);
    n.c = lds_ld4(q + 2);
    const float4 d = lds_ld4(q + 3);
    n.d = make_int4(__builtin_bit_cast(int, d.x), __builtin_bit_cast(int, d.y), __builtin_bit_cast(int, d.z),
                    __builtin_bit_cast(int, d.w));
    return n;
}
RR_D TriPack load_tri(const TriPack* __restrict__ p, int i) { return p[i]; }
RR_D TriPack load_tri(lds_tri* p, int i) {
    const __attribute__((address_space(3))) rr_f4v* q = (const __attribute__((address_space(3))) rr_f4v*)(p + i);
    TriPack t;
    t.p0 = lds_ld4(q);
    t.p1 = lds_ld4(q + 1);
    t.p2 = lds_ld4(q + 2);
    return t;
}
// kB: the threads per block of the kernel that owns the stack; kL: its LDS
// entries per lane (rr_debug_trace width 6 runs the 6-wide walk with 1, so
// nearly every entry lives in the HBM part); kS: its HBM entries per lane.
template <int kB = kBlock, int kL = kLdsStack, int kS = kSpillStack>
struct TravStackT {
    // Bases only: the lane's slots are recomputed from threadIdx/blockIdx at each
    // push/pop, so no per-lane pointer stays live in VGPRs across a kernel's
    // ray loop.
    lds_int* lds;   // lds_base: lane slot lds[sp * kB + threadIdx.x]
    int* spill;     // spill_base: lane slot spill[(sp - kL) * stride + global thread]
    int spill_stride;
    int sp;
    // the frame's drop counter (device.hpp drops_slot; null: not counted)
    uint32_t* drops;
    // A push beyond kL + kS entries is dropped (a missed
    // subtree) and counted at once with an atomic on the frame's drop counter
    // (no register stays live for it; rr_frame_stats.stack_drops, tests assert
    // 0 on every bench scene); the oracle's stack has the same capacity and the
    // same rule (ORC_MAXDEPTH) and counts its drops too (orc_stack_drops).
    RR_D void push(int x) {
        if (sp < kL) {
            lds[sp * kB + (int)threadIdx.x] = x;
        } else if (sp < kL + kS) {
            spill[(sp - kL) * spill_stride + (int)(blockIdx.x * kB + threadIdx.x)] = x;
        } else {
            if (drops) atomicAdd(drops, 1u);
            return;
        }
        ++sp;
    }
    RR_D int pop() {
        --sp;
        if (sp < kL) return lds[sp * kB + (int)threadIdx.x];
        return spill[(sp - kL) * spill_stride + (int)(blockIdx.x * kB + threadIdx.x)];
    }
    // Grouped entries of the 6-wide walk (RR_STACK_GROUP): one entry per node
    // for all the internal children it leaves for later, first child index << 6
    // | the mask of their ranks among the node's internal children (internal
    // children are consecutive nodes: child of rank k = first + k). pop_group
    // takes the lowest rank and keeps the entry while ranks remain, so the
    // children come off in the order single pushes in descending slot order
    // gave (the walk visits the same nodes in the same order).
    RR_D int pop_group() {
        const int i = sp - 1;
        const bool in_lds = i < kL;
        const int gi = (i - kL) * spill_stride + (int)(blockIdx.x * kB + threadIdx.x);
        const int e = in_lds ? lds[i * kB + (int)threadIdx.x] : spill[gi];
        const int node = (int)((uint32_t)e >> 6) + __builtin_ctz((uint32_t)e & 63u);
        const int rest = e & (e - 1);  // the lowest rank bit cleared
        if ((rest & 63) == 0) {
            sp = i;
        } else if (in_lds) {
            lds[i * kB + (int)threadIdx.x] = rest;
        } else {
            spill[gi] = rest;
        }
        return node;
    }
};
// The ranks among a node's internal children (imask) of the internal slots in
// rest (a subset of imask), as a mask: bit k = the internal child of rank k.
RR_D uint32_t q6_rank_mask(uint32_t rest, uint32_t imask) {
    uint32_t r = 0, k = 0;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        r |= ((rest >> c) & 1u) << k;
        k += (imask >> c) & 1u;
    }
    return r;
}
// RR_STACK_GROUP (default): the 6-wide walks push one grouped entry per node
// (pop_group) instead of one entry per child: per 02 / 03 / C5 frame slice
// 80.5 / 86.7 / 69.6 -> 79.0 / 85.5 / 69.3 ms (profiles/r5_ab_walk.txt). The
// oracle's walk keeps the same entries, so both stacks fill (and drop) alike.
#ifndef RR_STACK_GROUP
#define RR_STACK_GROUP 1
#endif
using TravStack = TravStackT<kBlock>;

RR_D lds_int* lds_slot(int* shared_elem) {
    return (lds_int*)(shared_elem);
}

// Traversal counters for RR_FLAG_COUNT_TRAVERSAL builds (kCount = true only).
struct TravCount {
    uint32_t nodes = 0, tris = 0;
};

// Resumable traversal of one ray: start() then step() until it returns true.
// Near child first (left on ties); leaf children are intersected as soon as
// their box passes. The fused path kernels run it to completion per lane
// (traverse() below); the split trace kernels of large scenes interleave
// step() with lane refill (wavefront.hip trace_refill), which changes only the
// schedule, never the visited nodes, so the hits are identical.
// nodes / tris: global or LDS pointers (wavefront.hip SceneView).
// The largest |coordinate| of a BVH2's scene box (its root's two child boxes).
RR_D float scene_radius(const BvhNode& r) {
    const float a = fmaxf(fmaxf(fmaxf(fabsf(r.a.x), fabsf(r.a.y)), fmaxf(fabsf(r.a.z), fabsf(r.a.w))),
                          fmaxf(fabsf(r.b.x), fabsf(r.b.y)));
    const float b = fmaxf(fmaxf(fmaxf(fabsf(r.b.z), fabsf(r.b.w)), fmaxf(fabsf(r.c.x), fabsf(r.c.y))),
                          fmaxf(fabsf(r.c.z), fabsf(r.c.w)));
    return fmaxf(a, b);
}

template <bool kAnyHit, bool kCount = false>
struct TravState {
    float3 o, invd, oi, em;
    Shear sh;
    float tmin;
    Hit h;
    int node;
    // r: scene_radius of the hierarchy walked (the box margins, slab_margin)
    RR_D void start(float3 o_, float3 d_, float tmin_, float tmax_, float r) {
        o = o_;
        sh = make_shear(d_);
        tmin = tmin_;
        h.t = tmax_;
        h.u = h.v = 0.0f;
        h.idx = -1;
        h.orig = -1;
        invd = rcp3(d_);
        oi = mk3(-(o.x * invd.x), -(o.y * invd.y), -(o.z * invd.z));
        em = slab_margin(o, invd, r);
        node = 0;
    }
    // One node visit; true when the ray is finished (any-hit: on the first hit).
    template <typename NodeP, typename TriP, typename Stack>
    RR_D bool step(NodeP nodes, TriP tris, Stack& st, TravCount& cnt) {
        const BvhNode nd = load_node(nodes, node);
        if (kCount) ++cnt.nodes;
        float tl, tr;
        bool hl = slab(oi, invd, em, nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y, tmin, h.t, tl);
        bool hr = slab(oi, invd, em, nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w, tmin, h.t, tr);
        const int cl = nd.d.x, cr = nd.d.y;
        // passing leaves (single triangles), left then right, one per
        // iteration: lanes with only a left and lanes with only a right leaf
        // share one pass, a wave runs as many passes as its busiest lane needs
        int nl = 0, nr = 0;
        if (hl && cl < 0) {
            nl = 1;
            hl = false;
        }
        if (hr && cr < 0) {
            nr = 1;
            hr = false;
        }
        for (int k = 0; k < nl + nr; ++k) {
            const int ti = k < nl ? ~cl : ~cr;
            if (kCount) ++cnt.tris;
            leaf_test(load_tri(tris, ti), ti, sh, o, tmin, h);
            if (kAnyHit && h.idx >= 0) return true;
        }
        if (hl && hr) {
            const bool left_first = tl <= tr;
            st.push(left_first ? cr : cl);
            node = left_first ? cl : cr;
        } else if (hl) {
            node = cl;
        } else if (hr) {
            node = cr;
        } else {
            if (st.sp == 0) return true;
            node = st.pop();
        }
        return false;
    }
};

// Per-node terms of the quantised box tests for one ray (iq: rcp3 of the
// direction). Per axis s = iq * 2^e (exact); a plane at grid coordinate q lies
// at t = fma(q, s, (org - o) * iq), the near planes' offsets less the axis'
// margin m |iq|, the far planes' more, folded into one fma each, so a box
// holding a triangle woop_test accepts is never rejected by rounding. The
// margin distance m = kBoxMargin (the largest |org - o| + 255 * 2^(the largest
// e)): the node's own distance from the origin plus its extent bound every
// plane distance of its children and every vertex below it, so the rounding
// of both tests stays under it (the largest exponent is stored in the node,
// so the bound costs a max, an ldexp and an fma). (A per-ray bound, kBoxMargin (|o|_inf + twice
// the root grid's largest |coordinate|), saved 8 VALU per node visit but was
// loose deep in the tree: 3.7 % more triangle tests on C5 bounce rays, and
// measured 1 / 1 / 3.4 % slower on 02 / 03 / C5 frame slices.)
struct Q6Planes {
    float sx, sy, sz;     // iq * 2^e
    float nx, ny, nz;     // (org - o) iq - margin (near planes)
    float fx, fy, fz;     // (org - o) iq + margin (far planes)
};
// org: the node's grid origin and exponent word (QNode6::org), cw: its
// used-slot word (QNode6::c.w: the largest exponent in bits 8..15).
RR_D Q6Planes q6_planes_of(float4 org, uint32_t cw, float3 o, float3 iq) {
    const uint32_t eb = (uint32_t)f2i(org.w);
    const int ex = (int)(eb & 255u) - 128, ey = (int)((eb >> 8) & 255u) - 128, ez = (int)((eb >> 16) & 255u) - 128;
    const float dx = org.x - o.x, dy = org.y - o.y, dz = org.z - o.z;
    // (the largest |org - o| + 255 * 2^(the largest e, kept in c.w bits 8..15))
    // kBoxMargin: at least the per-axis maximum of |org - o| + extent
    const float m = fmaf(fmaxf(fmaxf(fabsf(dx), fabsf(dy)), fabsf(dz)), kBoxMargin,
                         ldexpf(255.0f * kBoxMargin, (int)((cw >> 8) & 255u) - 128));
    const float3 em = mk3(m * fabsf(iq.x), m * fabsf(iq.y), m * fabsf(iq.z));
    Q6Planes p;
    p.sx = ldexpf(iq.x, ex);
    p.sy = ldexpf(iq.y, ey);
    p.sz = ldexpf(iq.z, ez);
    p.nx = fmaf(dx, iq.x, -em.x);
    p.ny = fmaf(dy, iq.y, -em.y);
    p.nz = fmaf(dz, iq.z, -em.z);
    p.fx = fmaf(dx, iq.x, em.x);
    p.fy = fmaf(dy, iq.y, em.y);
    p.fz = fmaf(dz, iq.z, em.z);
    return p;
}
RR_D Q6Planes q6_planes(const QNode6& n, float3 o, float3 iq) { return q6_planes_of(n.org, n.c.w, o, iq); }

// The six child box tests of a quantised node for one ray: bit c set when
// child c's box meets [tmin, tcur] (never for an unused slot: the used-slot
// mask in c.w is applied, which also holds when a NaN ray component makes
// fmaxf / fminf drop their operands); tn[c] = the entry distance. The near
// plane is lo for iq >= 0, else hi (iq is never 0 or inf, so no NaN and no
// min/max per axis). oracle/rr_oracle.c trace4() restates it.
RR_D uint32_t q6_box_hits(const QNode6& n, float3 o, float3 iq, float tmin, float tcur, float tn[kQWidth]) {
    const Q6Planes pl = q6_planes(n, o, iq);
    const float sx = pl.sx, sy = pl.sy, sz = pl.sz;
    const bool px = iq.x >= 0.0f, py = iq.y >= 0.0f, pz = iq.z >= 0.0f;
    // children 0..3: one byte each of the near / far words per axis
    const uint32_t nx = px ? n.a.z : n.b.y, fx = px ? n.b.y : n.a.z;
    const uint32_t ny = py ? n.a.w : n.b.z, fy = py ? n.b.z : n.a.w;
    const uint32_t nz = pz ? n.b.x : n.b.w, fz = pz ? n.b.w : n.b.x;
    // children 4, 5: the byte pairs in the low / high halves of c.x .. c.z
    const uint32_t lox = n.c.x & 0xffffu, loy = n.c.x >> 16, loz = n.c.y & 0xffffu;
    const uint32_t hix = n.c.y >> 16, hiy = n.c.z & 0xffffu, hiz = n.c.z >> 16;
    const uint32_t nx2 = px ? lox : hix, fx2 = px ? hix : lox;
    const uint32_t ny2 = py ? loy : hiy, fy2 = py ? hiy : loy;
    const uint32_t nz2 = pz ? loz : hiz, fz2 = pz ? hiz : loz;
    uint32_t hits = 0;
#pragma unroll
    for (int c = 0; c < kQWidth; ++c) {
        const int sh = c < 4 ? 8 * c : 8 * (c - 4);
        const uint32_t qnx = c < 4 ? nx : nx2, qny = c < 4 ? ny : ny2, qnz = c < 4 ? nz : nz2;
        const uint32_t qfx = c < 4 ? fx : fx2, qfy = c < 4 ? fy : fy2, qfz = c < 4 ? fz : fz2;
        const float t0 = fmaxf(fmaxf(fmaf((float)((qnx >> sh) & 255u), sx, pl.nx), fmaf((float)((qny >> sh) & 255u), sy, pl.ny)),
                               fmaxf(fmaf((float)((qnz >> sh) & 255u), sz, pl.nz), tmin));
        const float t1 = fminf(fminf(fmaf((float)((qfx >> sh) & 255u), sx, pl.fx), fmaf((float)((qfy >> sh) & 255u), sy, pl.fy)),
                               fminf(fmaf((float)((qfz >> sh) & 255u), sz, pl.fz), tcur));
        tn[c] = t0;
        if (t0 <= t1) hits |= 1u << c;
    }
    return hits & n.c.w;
}

// q6_box_hits that keeps only the nearest hit internal child (ties: lower
// slot) instead of every entry distance: six fewer live registers in the
// per-lane walk (TravStateQ6); best = -1 when no internal child is hit.
// kNearest false (any-hit rays): the lowest hit internal slot instead. An
// any-hit walk opens every node whose box meets [tmin, tmax] until its first
// hit (the bound never shrinks), so the order decides nothing but the speed:
// slot order drops the distance compares and their registers (shadow rays
// -10 % on C5, VGPR spill slots 10 -> 2).
template <bool kNearest = true>
RR_D uint32_t q6_box_best(const QNode6& n, float3 o, float3 iq, float tmin, float tcur, uint32_t imask,
                          int& best) {
    const Q6Planes pl = q6_planes(n, o, iq);
    const float sx = pl.sx, sy = pl.sy, sz = pl.sz;
    const uint32_t used = n.c.w;
    const bool px = iq.x >= 0.0f, py = iq.y >= 0.0f, pz = iq.z >= 0.0f;
    const uint32_t nx = px ? n.a.z : n.b.y, fx = px ? n.b.y : n.a.z;
    const uint32_t ny = py ? n.a.w : n.b.z, fy = py ? n.b.z : n.a.w;
    const uint32_t nz = pz ? n.b.x : n.b.w, fz = pz ? n.b.w : n.b.x;
    const uint32_t lox = n.c.x & 0xffffu, loy = n.c.x >> 16, loz = n.c.y & 0xffffu;
    const uint32_t hix = n.c.y >> 16, hiy = n.c.z & 0xffffu, hiz = n.c.z >> 16;
    const uint32_t nx2 = px ? lox : hix, fx2 = px ? hix : lox;
    const uint32_t ny2 = py ? loy : hiy, fy2 = py ? hiy : loy;
    const uint32_t nz2 = pz ? loz : hiz, fz2 = pz ? hiz : loz;
    // The used-slot mask is applied once at the end; the best-slot choice
    // needs none (internal slots are used slots). bt starts at +inf: the entry
    // distance of a hit box is finite (t0 <= t1 <= tcur).
    uint32_t hits = 0;
    best = -1;
    float bt = __builtin_inff();
#pragma unroll
    for (int c = 0; c < kQWidth; ++c) {
        const int sh = c < 4 ? 8 * c : 8 * (c - 4);
        const uint32_t qnx = c < 4 ? nx : nx2, qny = c < 4 ? ny : ny2, qnz = c < 4 ? nz : nz2;
        const uint32_t qfx = c < 4 ? fx : fx2, qfy = c < 4 ? fy : fy2, qfz = c < 4 ? fz : fz2;
        const float t0 = fmaxf(fmaxf(fmaf((float)((qnx >> sh) & 255u), sx, pl.nx), fmaf((float)((qny >> sh) & 255u), sy, pl.ny)),
                               fmaxf(fmaf((float)((qnz >> sh) & 255u), sz, pl.nz), tmin));
        const float t1 = fminf(fminf(fmaf((float)((qfx >> sh) & 255u), sx, pl.fx), fmaf((float)((qfy >> sh) & 255u), sy, pl.fy)),
                               fminf(fmaf((float)((qfz >> sh) & 255u), sz, pl.fz), tcur));
        const bool hit = t0 <= t1;
        hits |= (uint32_t)hit << c;
        if (hit && ((imask >> c) & 1u) && (!kNearest ? best < 0 : t0 < bt)) {
            best = c;
            bt = t0;
        }
    }
    return hits & used;
}

// Node fetch of the 6-wide walk. The split-path trace kernels keep a copy of
// the first n_top nodes in LDS (Q6Nodes): nodes are numbered breadth first,
// so those are the top levels of the tree, which every ray visits — each of
// those visits becomes a ds_read instead of an L2 round trip. Which copy a
// node comes from changes no bit of it.
RR_D QNode6 q6_load(const QNode6* __restrict__ nodes, int i) { return nodes[i]; }
struct Q6Nodes {
    const QNode6* __restrict__ g;
    lds_f4w* top;  // nodes [0, n_top): 4 float4 each (QNode6 layout)
    int n_top;
};
RR_D uint4 f4_bits(float4 v) {
    return make_uint4((uint32_t)f2i(v.x), (uint32_t)f2i(v.y), (uint32_t)f2i(v.z), (uint32_t)f2i(v.w));
}
// RR_FLAT_TOP (default): per 02 / 03 / C5 frame slice 78.5 / 85.0 / 69.1 ->
// 78.4 / 84.8 / 68.7 ms (profiles/r5_ab_lds.txt; the branchy form measured
// within 0.5 % of it, and the 4 x 16 B of a node arrive either way).
#ifndef RR_FLAT_TOP
#define RR_FLAT_TOP 1
#endif
RR_D QNode6 q6_load(const Q6Nodes& n, int i) {
#if RR_FLAT_TOP
    // one generic (flat) pointer for both copies: a wave whose lanes read
    // both takes one set of loads, not the two branches in turn (where the LDS
    // reads waited for the HBM loads, whose registers they reuse)
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v* top_g = (const u4v*)(const rr_f4v*)n.top;
    const u4v* q = i < n.n_top ? top_g + 4 * i : reinterpret_cast<const u4v*>(n.g + i);
    const u4v w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    QNode6 r;
    r.org = make_float4(__uint_as_float(w0.x), __uint_as_float(w0.y), __uint_as_float(w0.z), __uint_as_float(w0.w));
    r.a = make_uint4(w1.x, w1.y, w1.z, w1.w);
    r.b = make_uint4(w2.x, w2.y, w2.z, w2.w);
    r.c = make_uint4(w3.x, w3.y, w3.z, w3.w);
    return r;
#endif
    if (i < n.n_top) {
        const lds_f4w* q = n.top + 4 * i;
        QNode6 r;
        r.org = lds_ld4(q);
        r.a = f4_bits(lds_ld4(q + 1));
        r.b = f4_bits(lds_ld4(q + 2));
        r.c = f4_bits(lds_ld4(q + 3));
        return r;
    }
    return q6_load(n.g, i);
}

// Resumable traversal of the quantised 6-wide hierarchy (same contract as
// TravState), box tests by q6_box_best. Leaf children whose boxes pass are
// intersected at once in slot order; the nearest hit internal child (any-hit
// rays: the lowest hit internal slot) is visited next and the others are
// pushed in descending slot order.
// oracle/rr_oracle.c trace4() is the same walk.
template <bool kAnyHit, bool kCount = false>
struct TravStateQ6 {
    float3 o, iq;
    Shear sh;
    float tmin;
    Hit h;
    int node;
    // (no scene radius, unlike TravState::start: the margins are per node, q6_planes)
    RR_D void start(float3 o_, float3 d_, float tmin_, float tmax_) {
        o = o_;
        sh = make_shear(d_);
        tmin = tmin_;
        h.t = tmax_;
        h.u = h.v = 0.0f;
        h.idx = -1;
        h.orig = -1;
        iq = rcp3(d_);
        node = 0;
    }
    template <typename NodeSrc, typename TriP, typename Stack>
    RR_D bool step(const NodeSrc& nodes, TriP tris, Stack& st, TravCount& cnt) {
        if (kCount) ++cnt.nodes;
        const float tcur = h.t;
        const auto nd = q6_load(nodes, node);
        const uint32_t imask = q6_inner(nd);
        int best;
        const uint32_t hm = q6_box_best<!kAnyHit>(nd, o, iq, tmin, tcur, imask, best);
        uint32_t leaves = hm & ~imask;
        const uint32_t inner = hm & imask;
        // passing leaves in slot order; the loop runs as often as the lane with
        // the most leaves needs, not once per slot
        while (leaves) {
            const int c = __builtin_ctz(leaves);
            leaves &= leaves - 1;
            const int ti = q6_first_leaf(nd) + c - __builtin_popcount(imask & ((1u << c) - 1u));
            if (kCount) ++cnt.tris;
            leaf_test(load_tri(tris, ti), ti, sh, o, tmin, h);
            if (kAnyHit && h.idx >= 0) return true;
        }
        if (!inner) {
            if (st.sp == 0) return true;
            node = RR_STACK_GROUP ? st.pop_group() : st.pop();
            return false;
        }
        // nearest hit child next (ties: lower slot, q6_box_best); the other hit
        // children are pushed in descending slot order (so they pop in slot order)
        const uint32_t rest = inner & ~(1u << best);
        const int base = q6_first_inner(nd);
#if RR_STACK_GROUP
        if (rest) st.push((int)(((uint32_t)base << 6) | q6_rank_mask(rest, imask)));
#else
#pragma unroll
        for (int c = kQWidth - 1; c >= 0; --c)
            if ((rest >> c) & 1u) st.push(base + __builtin_popcount(imask & ((1u << c) - 1u)));
#endif
        node = base + __builtin_popcount(imask & ((1u << best) - 1u));
        return false;
    }
};

// TravStateQ6 with postponed leaf tests (Aila & Laine 2009, "while-while"):
// a node visit records the leaf children its ray enters (slot mask, the node's
// first leaf triangle and internal-slot mask) instead of testing them, and the
// lane then waits; the wave runs its leaf tests together, one triangle per
// pending lane per step, once at least kLeafPhase of the lanes calling step()
// have leaves pending (or every one has). With immediate tests, the leaf loop
// ran as often as the lane with the most entered leaves needed while the
// others idled (0.46 of the lanes active per VALU instruction on C5). A lane
// with pending leaves visits no node until they are tested, so the closest-hit
// bound every box test uses is the same as with immediate tests: the same
// nodes are visited, the same triangles tested, only in another interleaving
// across lanes, and the accept rule makes the hit the same (bit-exact).
#ifndef RR_LEAF_PHASE
#define RR_LEAF_PHASE 12
#endif
#ifndef RR_LEAF_PHASE_ANY
#define RR_LEAF_PHASE_ANY RR_LEAF_PHASE  // the any-hit (shadow) walks' threshold
#endif
template <bool kAnyHit, bool kCount = false>
struct TravStateQ6D {
    float3 o, iq;
    Shear sh;
    float tmin;
    Hit h;
    int node;        // next node to visit, -1: none (the walk ends once the pending leaves are tested)
    int lbase;       // pending leaves: the node's first leaf triangle
    uint32_t lmask;  // pending leaf slots (bits 0..5) | the node's internal-slot mask << 8; 0: none
    RR_D void start(float3 o_, float3 d_, float tmin_, float tmax_) {
        o = o_;
        sh = make_shear(d_);
        tmin = tmin_;
        h.t = tmax_;
        h.u = h.v = 0.0f;
        h.idx = -1;
        h.orig = -1;
        iq = rcp3(d_);
        node = 0;
        lmask = 0;
    }
    template <typename NodeSrc, typename TriP, typename Stack>
    RR_D bool step(const NodeSrc& nodes, TriP tris, Stack& st, TravCount& cnt) {
        const uint64_t act = __ballot(true), pen = __ballot((lmask & 63u) != 0u);
        if (pen != 0 && (pen == act || __popcll(pen) >= (kAnyHit ? RR_LEAF_PHASE_ANY : RR_LEAF_PHASE))) {  // leaf phase
            if ((lmask & 63u) == 0u) return false;
            const int c = __builtin_ctz(lmask);
            lmask &= lmask - 1u;
            const uint32_t imask = lmask >> 8;
            const int ti = lbase + c - __builtin_popcount(imask & ((1u << c) - 1u));
            if (kCount) ++cnt.tris;
            leaf_test(load_tri(tris, ti), ti, sh, o, tmin, h);
            if (kAnyHit && h.idx >= 0) return true;
            if ((lmask & 63u) == 0u) lmask = 0u;
            return lmask == 0u && node < 0;
        }
        if (lmask != 0u) return false;  // waits for the leaf phase
        if (kCount) ++cnt.nodes;
        const float tcur = h.t;
        const auto nd = q6_load(nodes, node);
        const uint32_t imask = q6_inner(nd);
        int best;
        const uint32_t hm = q6_box_best<!kAnyHit>(nd, o, iq, tmin, tcur, imask, best);
        const uint32_t leaves = hm & ~imask;
        const uint32_t inner = hm & imask;
        if (leaves) {
            lbase = q6_first_leaf(nd);
            lmask = leaves | (imask << 8);
        }
        if (!inner) {
            if (st.sp == 0) {
                node = -1;
                return lmask == 0u;
            }
            node = RR_STACK_GROUP ? st.pop_group() : st.pop();
            return false;
        }
        const uint32_t rest = inner & ~(1u << best);
        const int base = q6_first_inner(nd);
#if RR_STACK_GROUP
        if (rest) st.push((int)(((uint32_t)base << 6) | q6_rank_mask(rest, imask)));
#else
#pragma unroll
        for (int c = kQWidth - 1; c >= 0; --c)
            if ((rest >> c) & 1u) st.push(base + __builtin_popcount(imask & ((1u << c) - 1u)));
#endif
        node = base + __builtin_popcount(imask & ((1u << best) - 1u));
        return false;
    }
};

// Closest hit (or any hit) over the LBVH, run to completion.
template <bool kAnyHit, bool kCount = false, typename NodeP, typename TriP, typename Stack>
RR_D bool traverse(NodeP nodes, TriP tris, int n_tris, float3 o, float3 d, float tmin, float tmax, Stack& st, Hit& h,
                   TravCount& cnt) {
    if (n_tris <= 0) {  // the miss TravState::start would leave, without its three divisions
        h.t = tmax;
        h.u = h.v = 0.0f;
        h.idx = -1;
        h.orig = -1;
        return false;
    }
    TravState<kAnyHit, kCount> ts;
    ts.start(o, d, tmin, tmax, scene_radius(load_node(nodes, 0)));
    st.sp = 0;
    while (!ts.step(nodes, tris, st, cnt)) {
    }
    h = ts.h;
    return h.idx >= 0;
}

// ------------------------------------------------------------ materials ---
// Blender 3.6 Cycles' Principled BSDF (v1) for the subset the scenes use:
// base colour, metallic, specular, roughness (no transmission, clearcoat,
// sheen, subsurface, anisotropy or specular tint). Restated from Cycles'
// closure setup (intern/cycles/kernel/svm/closure.h, NODE_CLOSURE_BSDF /
// CLOSURE_BSDF_PRINCIPLED_ID), bsdf_principled_diffuse.h
// (PRINCIPLED_DIFFUSE_FULL) and the GGX-with-Fresnel microfacet closure
// (bsdf_microfacet.h, interpolate_fresnel_color / fresnel_dielectric_cos in
// bsdf_util.h); Cycles is third-party and not in the reference tree, so this
// restatement is unpinned against Cycles' own output.
//
// The two functions of a material that need a square root and two divisions
// each — Cycles' Fresnel blend FH and the specular-lobe pick probability —
// are tabulated per material on the host (build_material_lut, identical
// double-precision construction in the oracle) and read by linear
// interpolation: kMatLutN intervals over cos in [0, 1], FH against the cosine
// of the half angle, the pick probability against the cosine of the view
// angle (interpolation error below 4e-4 for specular IORs 1.2 .. 2).
constexpr int kMatLutN = 128;
constexpr int kMatLutStride = 260;  // floats per material: FH [0, 128] + repeat, ps [130, 258] + repeat
constexpr int kMatLutPs = 130;      // offset of the pick-probability channel

struct Mat {
    float3 base;
    float metallic, specular, roughness, ior;
    float3 emission;
    int model;  // 0 Principled subset, 1 pure Lambert (analytic test scenes)
    // per-material terms (mat_derive), evaluated once per material load
    float alpha, a2;   // GGX roughness alpha = max(roughness^2, 1e-3), alpha^2
    float3 cspec0;     // Cycles cspec0 = saturate(0.08 specular (1 - metallic) + base metallic)
    float kd0;         // (1 - metallic) / pi
    int spec_on;       // the specular closure exists (specular or metallic > 1e-5)
};

RR_HD float saturatef_(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

RR_HD void mat_derive(Mat& m) {
    // alpha floor 1e-3 (roughness 0.032): below it the float GGX terms break
    // down (a2 - 1 rounds to -1, D overflows at N.H = 1); Cycles switches to
    // a singular mirror lobe below alpha^2 = 1e-7 instead
    float alpha = m.roughness * m.roughness;
    if (alpha < 1.0e-3f) alpha = 1.0e-3f;
    m.alpha = alpha;
    m.a2 = alpha * alpha;
    const float sm = m.specular * 0.08f * (1.0f - m.metallic);
    m.cspec0 = mk3(saturatef_(sm + m.base.x * m.metallic), saturatef_(sm + m.base.y * m.metallic),
                   saturatef_(sm + m.base.z * m.metallic));
    m.kd0 = (1.0f - m.metallic) * 0.318309886183791f;
    m.spec_on = (m.specular > 1.0e-5f || m.metallic > 1.0e-5f) ? 1 : 0;
}

RR_HD float schlick_w(float c) {
    float m = 1.0f - c;
    if (m < 0.0f) m = 0.0f;
    const float m2 = m * m;
    return m2 * m2 * m;
}

// A material table channel at u in [0, 1] (t: global or LDS pointer); each
// channel's last entry is repeated (build_material_lut), so the branch-free
// read applies.
template <typename FloatP>
RR_HD float lut_at(FloatP t, float u) {
    return table_lerp_padded(t, kMatLutN + 1, fminf(fmaxf(u, 0.0f), 1.0f));
}

// Terms of the view direction shared by every evaluation at one shading point
// (NEE and the sampled continuation): computed once per shading point.
struct BsdfView {
    float cosV, ps, fv;
    float cv1;  // cosV + sqrt(a2 + (1 - a2) cosV^2): Smith G1(V) = 2 cosV / cv1
};

// f * cosL (the BSDF times the cosine of the light direction, Cycles'
// convention) and the combined one-sample-MIS pdf of the two closures (Cycles
// surface_shader_bsdf_eval: every closure evaluated, pdfs weighted by the
// closures' sample weights):
//   diffuse  base (1 - metallic) / pi * [(1 - FV/2)(1 - FL/2) + RR (FL + FV + FL FV (RR - 1))],
//            RR = roughness (L.V + 1)            (PRINCIPLED_DIFFUSE_FULL)
//   specular F * D G1(V) G1(L) / (4 cosV cosL), GGX D, separable Smith G1,
//            F = cspec0 (1 - FH) + FH, FH = the table at L.H
// with |V + L|^2 = 2 + 2 L.V, so (N.H)^2 = (cosV + cosL)^2 / (2 + 2 L.V) and
// (L.H)^2 = (1 + L.V) / 2 (no normalised half vector). One division: with
// den = 2 + 2 L.V, tt = (N.H)^2 (a2 - 1) + 1 = X / den, X = (cosV + cosL)^2
// (a2 - 1) + den, and G1(c) = 2c / c1, c1 = c + sqrt(a2 + (1 - a2) c^2):
//   D G1(V) / (4 cosV)           = a2 den^2 / (2 pi X^2 cv1)        (pdf_s)
//   D G1(V) G1(L) / (4 cosV)     = a2 den^2 cosL / (pi X^2 cv1 cl1)  (ks)
// lut: this material's table (kMatLutStride floats).
template <typename FloatP>
RR_HD float3 bsdf_eval_v(const Mat& m, FloatP lut, const BsdfView& vw, float3 N, float3 wo, float3 wi, float& pdf) {
    const float cosV = vw.cosV;
    const float cosL = dot3(N, wi);
    if (cosV <= 0.0f || cosL <= 0.0f) {
        pdf = 0.0f;
        return mk3(0.0f, 0.0f, 0.0f);
    }
    if (m.model == 1) {
        pdf = cosL * 0.318309886183791f;
        return scl3(m.base, pdf);
    }
    const float ps = vw.ps;
    const float lv = dot3(wi, wo);
    const float a2 = m.a2;
    // diffuse
    const float fl = schlick_w(cosL);
    const float fv = vw.fv;
    const float rr = m.roughness * (lv + 1.0f);
    const float kd =
        m.kd0 * fmaf(rr, fmaf(fl * fv, rr - 1.0f, fl + fv), fmaf(-0.5f, fv, 1.0f) * fmaf(-0.5f, fl, 1.0f)) * cosL;
    // specular
    const float sv = cosV + cosL;
    const float den = fmaf(2.0f, lv, 2.0f);
    const float X = fmaf(sv * sv, a2 - 1.0f, den);
    // sqrt_rn arguments: a2 + (1 - a2) c^2 with c in (0, 1] lies between a2 >= 1e-6
    // (alpha floor) and 1; (1 + L.V) / 2 of unit vectors is 0, a multiple of
    // 2^-26 or a rounding below 0 (NaN on both sides, clamped to the table's
    // first entry by lut_at)
    const float cl1 = cosL + sqrt_rn(fmaf((1.0f - a2) * cosL, cosL, a2));
    const float q = a2 * den * den;
    const float r = 1.0f / (3.14159265358979f * X * X * vw.cv1 * cl1);
    const float pdf_s = q * cl1 * r * 0.5f;                 // D G1(V) / (4 cosV)
    const float ks = m.spec_on ? q * cosL * r : 0.0f;       // D G1(V) G1(L) / (4 cosV cosL) * cosL
    const float fh = lut_at(lut, sqrt_rn(fmaf(0.5f, lv, 0.5f)));  // L.H = sqrt((1 + L.V) / 2)
    const float3 c0 = m.cspec0;
    const float fh1 = 1.0f - fh;
    const float3 F = mk3(fmaf(c0.x, fh1, fh), fmaf(c0.y, fh1, fh), fmaf(c0.z, fh1, fh));
    const float pdf_d = cosL * 0.318309886183791f;
    pdf = fmaf(ps, pdf_s, (1.0f - ps) * pdf_d);
    return mk3(fmaf(F.x, ks, m.base.x * kd), fmaf(F.y, ks, m.base.y * kd), fmaf(F.z, ks, m.base.z * kd));
}

template <typename FloatP>
RR_HD BsdfView bsdf_view(const Mat& m, FloatP lut, float3 N, float3 wo) {
    BsdfView v;
    v.cosV = dot3(N, wo);
    v.ps = lut_at(lut + kMatLutPs, v.cosV);  // 0 for Lambert and without a specular closure
    v.fv = schlick_w(v.cosV);
    const float a2 = m.a2;
    v.cv1 = v.cosV + sqrt_rn(fmaf((1.0f - a2) * v.cosV, v.cosV, a2));  // >= a2 >= 1e-6 (as cl1)
    return v;
}

// The one-shot form (tests / inspection): same result as bsdf_eval_v with
// bsdf_view(m, lut, N, wo), except that the caller's ps is used.
template <typename FloatP>
RR_HD float3 bsdf_eval(const Mat& m, FloatP lut, float3 N, float3 wo, float3 wi, float ps, float& pdf) {
    BsdfView v = bsdf_view(m, lut, N, wo);
    v.ps = ps;
    return bsdf_eval_v(m, lut, v, N, wo, wi, pdf);
}

// GGX visible-normal sample in the local frame (N = +z), by spherical caps
// (Dupuy & Benyoub 2023): in the stretched configuration the visible normals
// of the view vh are vh + c for c uniform on the cap z > -vh.z of the unit
// sphere. (dx, dy): concentric_disk(u1, u2) (r^2 = dx^2 + dy^2 uniform, the
// angle uniform), drawn by the caller (bsdf_sample shares it between the
// lobes): z = 1 - r^2 (1 + vz), and (x, y) = (dx, dy) sqrt((1 + vz)(2 - r^2 (1 + vz)))
// so that x^2 + y^2 = 1 - z^2, without a division.
RR_HD float3 sample_vndf(float3 v, float alpha, float dx, float dy) {
    // |vh|^2 >= min(alpha^2, 1) |v|^2 with v a unit vector: sqrt_rn's range;
    // s^2 is 0 or a product of k >= 1 and a difference of 2 and an exact
    // product of floats of at most 2 (a multiple of 2^-48); the final h can
    // vanish at the cap's rim (sqrt_any)
    const float3 vh = norm3_rn(mk3(alpha * v.x, alpha * v.y, v.z));
    const float r2 = fmaf(dy, dy, dx * dx);
    const float k = 1.0f + vh.z;
    const float z = fmaf(-r2, k, 1.0f);
    const float s = sqrt_rn(fmaxf(0.0f, k * fmaf(-r2, k, 2.0f)));
    const float3 h = mk3(fmaf(dx, s, vh.x), fmaf(dy, s, vh.y), fmaxf(0.0f, z + vh.z));
    return norm3_any(mk3(alpha * h.x, alpha * h.y, h.z));
}

// Sample a direction; returns false when the path must end. f: f * cosL as
// bsdf_eval_v. glossy: the specular lobe was picked (Cycles LABEL_GLOSSY;
// else LABEL_DIFFUSE), which decides the bounce counter the scatter advances.
// (T, B): make_onb(N), which LDS-resident scenes stage per triangle side
// (wavefront.hip stage_scene) instead of computing it per sample.
template <typename FloatP>
RR_HD bool bsdf_sample_onb(const Mat& m, FloatP lut, const BsdfView& vw, float3 N, float3 T, float3 B, float3 wo,
                           float ul, float u1, float u2, float3& wi, float3& f, float& pdf, bool& glossy) {
    const float cosV = vw.cosV;
    if (cosV <= 0.0f) return false;
    const float ps = vw.ps;
    float x, y;  // the disk sample both lobes start from
    concentric_disk(u1, u2, x, y);
    glossy = ul < ps;
    // the lobe's direction in the local frame: the GGX half vector (glossy)
    // or the cosine-weighted point (diffuse); one frame3 for both, so a wave
    // whose lanes picked both lobes runs it once
    float3 l;
    if (glossy) {
        const float3 wl = mk3(dot3(wo, T), dot3(wo, B), cosV);
        l = sample_vndf(wl, m.alpha, x, y);
    } else {
        // 1 - x^2 - y^2 of a disk point: 0 or at least 2^-70 (sqrt_rn's range)
        l = mk3(x, y, sqrt_rn(fmaxf(0.0f, fmaf(-y, y, fmaf(-x, x, 1.0f)))));
    }
    const float3 W = frame3(T, B, N, l.x, l.y, l.z);
    if (glossy) {  // reflect wo about the half vector
        const float k = 2.0f * dot3(wo, W);
        wi = mk3(fmaf(W.x, k, -wo.x), fmaf(W.y, k, -wo.y), fmaf(W.z, k, -wo.z));
    } else {
        wi = W;
    }
    f = bsdf_eval_v(m, lut, vw, N, wo, wi, pdf);
    return pdf > 0.0f;
}
template <typename FloatP>
RR_HD bool bsdf_sample(const Mat& m, FloatP lut, const BsdfView& vw, float3 N, float3 wo, float ul, float u1,
                       float u2, float3& wi, float3& f, float& pdf, bool& glossy) {
    if (vw.cosV <= 0.0f) return false;
    float3 T, B;
    make_onb(N, T, B);
    return bsdf_sample_onb(m, lut, vw, N, T, B, wo, ul, u1, u2, wi, f, pdf, glossy);
}

RR_HD float3 clamp_contrib(float3 c, float clamp) {
    if (clamp > 0.0f) {
        const float mx = max3f(c);
        if (mx > clamp) return scl3(c, clamp / mx);
    }
    return c;
}

// sRGB OETF: linear segment below 0.0031308, host-built table above.
RR_HD float srgb_oetf(float x, const float* lut, int lut_n) {
    if (x <= 0.0031308f) return x * 12.92f;
    return table_lerp(lut, lut_n + 1, x);
}

RR_HD uint8_t quantize8(float f) {
    if (f <= 0.0f) return 0;
    if (f >= 1.0f) return 255;
    return (uint8_t)(f * 255.0f + 0.5f);
}

}  // namespace rr
