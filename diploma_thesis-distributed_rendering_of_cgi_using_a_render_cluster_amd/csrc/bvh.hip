// LBVH build on the device: K1 world transform + centroid
// bounds, K2 30-bit Morton codes, K3 stable 4x8-bit LSD radix sort, K4 Karras
// 2012 topology + bottom-up refit with arrival counters, K5 leaf-order
// triangle pack. Everything is integer or exact (min/max) except the world
// transform and the Morton quantisation, whose float ops are written in the
// same order as oracle/rr_oracle.c so the whole BVH is reproduced bit for bit.
//
// Replaces Cycles' BVH build inside bpy.ops.render.render
// (/root/reference/scripts/render-timing-script.py:90); the reference rebuilds
// the full Blender scene per frame, here only the per-frame rigid transforms are
// uploaded and the LBVH is rebuilt when they change.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstring>

#include "device.hpp"

namespace rr {

namespace {

constexpr int kSortItems = 4;                   // keys per thread
constexpr int kSortTile = kBlock * kSortItems;  // 1024 keys per block
constexpr int kScanTile = 1024;

__device__ __forceinline__ uint32_t f2o(float f) {  // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__device__ __forceinline__ float xf(const float* m, float x, float y, float z) {
    return m[0] * x + m[1] * y + m[2] * z + m[3];
}

// K1: object -> world, centroid sum (v0+v1)+v2 stored in the .w lanes,
// block min/max of the centroid sums folded into 6 ordered-uint words:
// slots 0..2 minima (start 0xFFFFFFFF), slots 3..5 maxima (start 0).
// (An earlier form stored -max as a minimum; hipcc 7.2's SLP packing of the
// decode into v_pk_add_f32 dropped one of the negations, so no float negation
// is left on this path.)
__global__ __launch_bounds__(kBlock) void k_transform(int n, const float4* __restrict__ local,
                                                      const int32_t* __restrict__ obj,
                                                      const float* __restrict__ xform,
                                                      float4* __restrict__ world,
                                                      uint32_t* __restrict__ bounds) {
    __shared__ uint32_t red[6];
    if (threadIdx.x < 6) red[threadIdx.x] = threadIdx.x < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    const int i = blockIdx.x * kBlock + threadIdx.x;
    uint32_t mn[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    if (i < n) {
        const float* m = xform + 12 * obj[i];
        float3 w[3];
        for (int k = 0; k < 3; ++k) {
            const float4 v = local[3 * i + k];
            w[k] = mk3(xf(m, v.x, v.y, v.z), xf(m + 4, v.x, v.y, v.z), xf(m + 8, v.x, v.y, v.z));
        }
        const float3 c = add3(add3(w[0], w[1]), w[2]);
        world[3 * i + 0] = make_float4(w[0].x, w[0].y, w[0].z, c.x);
        world[3 * i + 1] = make_float4(w[1].x, w[1].y, w[1].z, c.y);
        world[3 * i + 2] = make_float4(w[2].x, w[2].y, w[2].z, c.z);
        mn[0] = f2o(c.x); mn[1] = f2o(c.y); mn[2] = f2o(c.z);
        mn[3] = mn[0]; mn[4] = mn[1]; mn[5] = mn[2];
    }
    if (i < n) {
        for (int k = 0; k < 3; ++k) atomicMin(&red[k], mn[k]);
        for (int k = 3; k < 6; ++k) atomicMax(&red[k], mn[k]);
    }
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&bounds[threadIdx.x], red[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&bounds[threadIdx.x], red[threadIdx.x]);
}

// K2: 30-bit Morton code of the quantised centroid sum.
__global__ __launch_bounds__(kBlock) void k_morton(int n, const float4* __restrict__ world,
                                                   const uint32_t* __restrict__ bounds,
                                                   uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float lo[3] = {o2f(bounds[0]), o2f(bounds[1]), o2f(bounds[2])};
    const float hi[3] = {o2f(bounds[3]), o2f(bounds[4]), o2f(bounds[5])};
    const float c[3] = {world[3 * i].w, world[3 * i + 1].w, world[3 * i + 2].w};
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        const float s = ext > 0.0f ? 1024.0f / ext : 0.0f;
        float f = (c[k] - lo[k]) * s;
        f = fminf(fmaxf(f, 0.0f), 1023.0f);
        q[k] = (uint32_t)f;
    }
    keys[i] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    vals[i] = (uint32_t)i;
}

// K3a: per-block digit histogram, layout hist[digit * nblocks + block].
__global__ __launch_bounds__(kBlock) void k_radix_hist(int n, int shift, const uint32_t* __restrict__ keys,
                                                       uint32_t* __restrict__ hist, int nblocks) {
    __shared__ uint32_t cnt[256];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const int base = blockIdx.x * kSortTile;
    for (int k = 0; k < kSortItems; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

// K3b: stable scatter. Wave w owns keys [w*256, w*256+256) of the tile, walked
// in 4 rounds of 64; ranks within a round come from an 8-ballot digit match.
__global__ __launch_bounds__(kBlock) void k_radix_scatter(int n, int shift, const uint32_t* __restrict__ kin,
                                                          const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout,
                                                          uint32_t* __restrict__ vout,
                                                          const uint32_t* __restrict__ offs, int nblocks) {
    __shared__ uint32_t wcnt[4][256];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = 0; k < 4; ++k) wcnt[k][threadIdx.x] = 0;
    __syncthreads();
    const int base = blockIdx.x * kSortTile + w * 256;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t key[4], val[4], rank[4];
    bool ok[4];
    for (int r = 0; r < 4; ++r) {
        const int i = base + r * 64 + lane;
        ok[r] = i < n;
        key[r] = ok[r] ? kin[i] : 0u;
        val[r] = ok[r] ? vin[i] : 0u;
        const uint32_t d = (key[r] >> shift) & 255u;
        uint64_t peers = __ballot(ok[r]);
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t before = wcnt[w][d];
        rank[r] = before + (uint32_t)__popcll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        if (ok[r] && (peers & lt) == 0ull) wcnt[w][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {   // exclusive prefix over the 4 waves, per digit
        uint32_t s = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = wcnt[k][threadIdx.x];
            wcnt[k][threadIdx.x] = s;
            s += t;
        }
    }
    __syncthreads();
    for (int r = 0; r < 4; ++r) {
        if (!ok[r]) continue;
        const uint32_t d = (key[r] >> shift) & 255u;
        const uint32_t pos = offs[d * nblocks + blockIdx.x] + wcnt[w][d] + rank[r];
        kout[pos] = key[r];
        vout[pos] = val[r];
    }
}

// Block-wide exclusive scan helper for 1024 items (256 threads x 4).
__device__ uint32_t block_scan4(uint32_t v[4], uint32_t* lds_waves) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t t = v[0] + v[1] + v[2] + v[3];
    uint32_t inc = t;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
    }
    if (lane == 63) lds_waves[w] = inc;
    __syncthreads();
    uint32_t wave_off = 0, total = 0;
    for (int k = 0; k < 4; ++k) {
        if (k < w) wave_off += lds_waves[k];
        total += lds_waves[k];
    }
    uint32_t run = wave_off + inc - t;
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = v[k];
        v[k] = run;
        run += x;
    }
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(kBlock) void k_scan_tiles(int m, uint32_t* __restrict__ data,
                                                       uint32_t* __restrict__ part) {
    __shared__ uint32_t ws[4];
    const int base = blockIdx.x * kScanTile + threadIdx.x * 4;
    uint32_t v[4];
    for (int k = 0; k < 4; ++k) v[k] = (base + k < m) ? data[base + k] : 0u;
    const uint32_t total = block_scan4(v, ws);
    for (int k = 0; k < 4; ++k)
        if (base + k < m) data[base + k] = v[k];
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// Exclusive scan of the tile totals by one block (loops over 1024-item slabs).
__global__ __launch_bounds__(kBlock) void k_scan_parts(int np, uint32_t* __restrict__ part) {
    __shared__ uint32_t ws[4];
    uint32_t carry = 0;
    for (int s = 0; s < np; s += kScanTile) {
        const int base = s + threadIdx.x * 4;
        uint32_t v[4];
        for (int k = 0; k < 4; ++k) v[k] = (base + k < np) ? part[base + k] : 0u;
        const uint32_t total = block_scan4(v, ws);
        for (int k = 0; k < 4; ++k)
            if (base + k < np) part[base + k] = v[k] + carry;
        carry += total;
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_add(int m, uint32_t* __restrict__ data,
                                                     const uint32_t* __restrict__ part) {
    const int base = blockIdx.x * kScanTile + threadIdx.x * 4;
    const uint32_t add = part[blockIdx.x];
    for (int k = 0; k < 4; ++k)
        if (base + k < m) data[base + k] += add;
}

__device__ __forceinline__ int delta(const uint32_t* __restrict__ keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = keys[i], b = keys[j];
    if (a == b) return 32 + __clz((uint32_t)(i ^ j));
    return __clz(a ^ b);
}

// K4a: Karras 2012 topology of internal node i.
__global__ __launch_bounds__(kBlock) void k_karras(int n, const uint32_t* __restrict__ keys,
                                                   int2* __restrict__ children,
                                                   int32_t* __restrict__ node_parent,
                                                   int32_t* __restrict__ leaf_parent,
                                                   int2* __restrict__ range) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    int t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    int left, right;
    if (lo == gamma) {
        left = ~gamma;
        leaf_parent[gamma] = 2 * i;
    } else {
        left = gamma;
        node_parent[gamma] = 2 * i;
    }
    if (hi == gamma + 1) {
        right = ~(gamma + 1);
        leaf_parent[gamma + 1] = 2 * i + 1;
    } else {
        right = gamma + 1;
        node_parent[gamma + 1] = 2 * i + 1;
    }
    children[i] = make_int2(left, right);
    range[i] = make_int2(lo, hi - lo + 1);  // sorted leaves [lo, hi] under node i
    if (i == 0) node_parent[0] = -1;
}

__device__ __forceinline__ void st_agent(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}

// K4b + K5: pack leaf i, then climb. Boxes are handed between workgroups
// through agent-scope (write-through, L1-bypassing) stores/loads and a
// returning agent-scope arrival counter per node: the second arriver owns the
// node (MI355X_MICROARCH.md "Valid forms": sc1 stores drained before the
// counter add, sc1 loads after it).
__global__ __launch_bounds__(kBlock) void k_refit(int n, const uint32_t* __restrict__ order,
                                                  const float4* __restrict__ world,
                                                  const int32_t* __restrict__ tri_mat,
                                                  const int32_t* __restrict__ leaf_parent,
                                                  const int32_t* __restrict__ node_parent,
                                                  const int2* __restrict__ children,
                                                  uint32_t* __restrict__ flags,
                                                  BvhNode* __restrict__ nodes,
                                                  TriPack* __restrict__ tris) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int orig = (int)order[i];
    const float4 a = world[3 * orig], b = world[3 * orig + 1], c = world[3 * orig + 2];
    TriPack tp;
    tp.p0 = make_float4(a.x, a.y, a.z, i2f(orig));
    tp.p1 = make_float4(b.x, b.y, b.z, i2f(tri_mat[orig]));
    tp.p2 = make_float4(c.x, c.y, c.z, 0.0f);
    tris[i] = tp;
    float bx[6] = {fminf(fminf(a.x, b.x), c.x), fminf(fminf(a.y, b.y), c.y), fminf(fminf(a.z, b.z), c.z),
                   fmaxf(fmaxf(a.x, b.x), c.x), fmaxf(fmaxf(a.y, b.y), c.y), fmaxf(fmaxf(a.z, b.z), c.z)};
    if (n == 1) {  // single triangle: root with both children = leaf 0
        float* f = reinterpret_cast<float*>(&nodes[0]);
        for (int k = 0; k < 6; ++k) {
            f[k] = bx[k];
            f[6 + k] = bx[k];
        }
        nodes[0].d = make_int4(~0, ~0, 0, 0);
        return;
    }
    int penc = leaf_parent[i];
    for (int guard = 0; guard < 4096 && penc >= 0; ++guard) {
        const int p = penc >> 1, side = penc & 1;
        float* f = reinterpret_cast<float*>(&nodes[p]);
        for (int k = 0; k < 6; ++k) st_agent(f + 6 * side + k, bx[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t prev = __hip_atomic_fetch_add(&flags[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0u) return;  // first arrival: the sibling's thread finishes the node
        const int o = 6 * (1 - side);
        for (int k = 0; k < 3; ++k) bx[k] = fminf(bx[k], ld_agent(f + o + k));
        for (int k = 3; k < 6; ++k) bx[k] = fmaxf(bx[k], ld_agent(f + o + k));
        const int2 ch = children[p];
        int* fi = reinterpret_cast<int*>(f);
        __hip_atomic_store(fi + 12, ch.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fi + 13, ch.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fi + 14, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fi + 15, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        penc = node_parent[p];
    }
}

// ------------------------------------------------ 6-wide collapse ---
// The BVH2 (PLOC; Karras below 3 triangles) becomes the quantised 6-wide
// hierarchy of the split path (rr_device.h QNode6), top down, one level per
// launch pair:
//  - children of the node rooted at BVH2 node r: start from r's two children
//    (one slot for a one-triangle scene); a child that is a single triangle is
//    a leaf entry; while there are fewer than six entries, the internal entry
//    with the largest box measure (dx*dy + dy*dz + dz*dx, ties: lowest slot)
//    is opened (replaced by its left child, its right child appended);
//  - nodes are numbered breadth first and the internal children of a node
//    take consecutive indices in slot order (level frontier [lo, hi): node k
//    counts its internal children, an exclusive scan gives each node its
//    children's first index hi + prefix), so siblings share 128 B lines and a
//    node stores only the first index;
//  - the triangles of a node's leaf entries take consecutive positions of the
//    hierarchy's own triangle array (qtris, swapped into DevScene::tris after
//    the collapse) in slot order, after the triangles of the levels before and
//    of the nodes before it in its level (a second count and scan), so a node
//    stores only the first position and the mask of its internal slots;
//  - child boxes are quantised on the node's grid: origin = the lo corner of
//    the children's union, per axis the smallest exponent that spans it in
//    255 steps, lo rounded down and hi up (exactly, in double).
// oracle/rr_oracle.c lbvh_collapse4 / q4_pack restate it.
struct QwSet {
    int m;
    int ref[kQWidth];
    float lo[3][kQWidth], hi[3][kQWidth];
};

__device__ __forceinline__ float qw_measure(const QwSet& S, int c) {
    const float dx = S.hi[0][c] - S.lo[0][c], dy = S.hi[1][c] - S.lo[1][c], dz = S.hi[2][c] - S.lo[2][c];
    return dx * dy + dy * dz + dz * dx;
}

__device__ void qw_set(const BvhNode* __restrict__ nodes, int n, int r, QwSet& S) {
    auto put = [&](int slot, const BvhNode& nd, int side) {
        const float* f = reinterpret_cast<const float*>(&nd) + 6 * side;
        for (int a = 0; a < 3; ++a) {
            S.lo[a][slot] = f[a];
            S.hi[a][slot] = f[3 + a];
        }
        S.ref[slot] = n > 1 ? (side ? nd.d.y : nd.d.x) : ~0;
    };
    const BvhNode nd = nodes[r];
    put(0, nd, 0);
    put(1, nd, 1);
    S.m = n > 1 ? 2 : 1;  // one triangle: one leaf slot
    while (S.m < kQWidth) {
        int best = -1;
        float ba = 0.0f;
        for (int c = 0; c < S.m; ++c) {
            if (S.ref[c] < 0) continue;
            const float a = qw_measure(S, c);
            if (best < 0 || a > ba) {
                best = c;
                ba = a;
            }
        }
        if (best < 0) break;
        const BvhNode cn = nodes[S.ref[best]];
        put(S.m, cn, 1);
        put(best, cn, 0);
        ++S.m;
    }
}

// Level start: frontier [0, 1) = the BVH2 root, triangle positions from 0.
__global__ void k_qw_init(int32_t* __restrict__ ctl, int32_t* __restrict__ src) {
    ctl[0] = 0;
    ctl[1] = 1;
    ctl[2] = 0;
    src[0] = 0;
}

// cnt[k] = internal children, tcnt[k] = leaf children (one triangle each) of
// frontier node lo + k (0 past the frontier, k <= bound: the scans' totals
// land in [bound]).
__global__ __launch_bounds__(kBlock) void k_qw_count(const int32_t* __restrict__ ctl, int bound, int n,
                                                     const BvhNode* __restrict__ nodes,
                                                     const int32_t* __restrict__ src, uint32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ tcnt) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k > bound) return;
    const int lo = ctl[0], hi = ctl[1];
    uint32_t c = 0, t = 0;
    if (k < bound && lo + k < hi) {
        QwSet S;
        qw_set(nodes, n, src[lo + k], S);
        for (int j = 0; j < S.m; ++j) {
            if (S.ref[j] >= 0) ++c;
            else ++t;
        }
    }
    cnt[k] = c;
    tcnt[k] = t;
}

// Node lo + k: internal children -> indices hi + cnt[k] .., their BVH2 roots
// -> src; leaf entries -> triangle positions ctl[2] + tcnt[k] .. (after the
// exclusive scans), their triangles copied there; the quantised node -> out.
__global__ __launch_bounds__(kBlock) void k_qw_emit(const int32_t* __restrict__ ctl, int bound, int n,
                                                    const BvhNode* __restrict__ nodes, int32_t* __restrict__ src,
                                                    const uint32_t* __restrict__ cnt,
                                                    const uint32_t* __restrict__ tcnt,
                                                    const TriPack* __restrict__ tris, TriPack* __restrict__ qtris,
                                                    QNode6* __restrict__ out) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= bound) return;
    const int lo = ctl[0], hi = ctl[1];
    const int idx = lo + k;
    if (idx >= hi) return;
    QwSet S;
    qw_set(nodes, n, src[idx], S);
    const int inner_base = hi + (int)cnt[k], tri_base = ctl[2] + (int)tcnt[k];
    int next = inner_base, tpos = tri_base;
    uint32_t inner = 0u;
    for (int c = 0; c < S.m; ++c) {
        if (S.ref[c] >= 0) {
            src[next++] = S.ref[c];
            inner |= 1u << c;
        } else {
            qtris[tpos++] = tris[~S.ref[c]];
        }
    }
    // quantised child boxes: children 0..3 one byte per word, 4 and 5 in byte
    // pairs (rr_device.h QNode6)
    uint32_t w[9] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // lo x, lo y, lo z, hi x, hi y, hi z; pairs
    auto set_q = [&](int which, int c, uint32_t v) {
        if (c < 4) w[which] |= v << (8 * c);
        else w[6 + which / 2] |= v << (16 * (which & 1) + 8 * (c - 4));
    };
    float org[3];
    uint32_t eb = 0u;
    for (int a = 0; a < 3; ++a) {
        float l = S.lo[a][0], h = S.hi[a][0];
        for (int c = 1; c < S.m; ++c) {
            l = fminf(l, S.lo[a][c]);
            h = fmaxf(h, S.hi[a][c]);
        }
        const int e = q4_exponent((double)h - (double)l);
        org[a] = l;
        eb |= (uint32_t)(e + 128) << (8 * a);
        for (int c = 0; c < kQWidth; ++c) {
            set_q(a, c, c < S.m ? q4_quant(S.lo[a][c], l, e, false) : 255u);
            set_q(3 + a, c, c < S.m ? q4_quant(S.hi[a][c], l, e, true) : 0u);
        }
    }
    QNode6 o;
    o.org = make_float4(org[0], org[1], org[2], i2f((int)(eb | inner << 24)));
    o.a = make_uint4((uint32_t)inner_base, (uint32_t)tri_base, w[0], w[1]);
    o.b = make_uint4(w[2], w[3], w[4], w[5]);
    // used slots | the largest exponent byte << 8 (q6_planes' margin)
    const uint32_t emax = max(max(eb & 255u, (eb >> 8) & 255u), (eb >> 16) & 255u);
    o.c = make_uint4(w[6], w[7], w[8], ((1u << S.m) - 1u) | emax << 8);
    out[idx] = o;
}

// Next level: [hi, hi + total), triangle positions after this level's.
__global__ void k_qw_advance(int32_t* __restrict__ ctl, int bound, const uint32_t* __restrict__ cnt,
                             const uint32_t* __restrict__ tcnt) {
    const int hi = ctl[1];
    ctl[0] = hi;
    ctl[1] = hi + (int)cnt[bound];
    ctl[2] += (int)tcnt[bound];
}

// ------------------------------------------------------------------ PLOC ---
// Large scenes (split path) get a PLOC hierarchy (Meister & Bittner 2018,
// parallel locally-ordered clustering) instead of the Karras LBVH: starting
// from the Morton-sorted leaves, every cluster finds the neighbour within
// kPlocR positions whose merged box has the smallest surface measure
// (dx*dy + dy*dz + dz*dx; ties -> the lower position); mutual nearest
// neighbours merge into a new node, the survivors are compacted in order, and
// the rounds repeat until one cluster is left. Node indices are handed out
// downwards from n-2 in creation order (rank of the merge within its round),
// so the root — the last merge — is node 0. The result is a binary tree over
// the same leaves in the same BvhNode format, with fewer node visits per ray
// than the LBVH on scenes with uneven triangle sizes. oracle/rr_oracle.c
// ploc_build() is the same algorithm, operation for operation.
#ifndef RR_PLOC_R
#define RR_PLOC_R 16
#endif
constexpr int kPlocR = RR_PLOC_R;

// cluster k: cl[2k] = (lo.xyz, ref bits), cl[2k+1] = (hi.xyz, 0)
__device__ __forceinline__ float ploc_area(float4 alo, float4 ahi, float4 blo, float4 bhi) {
    const float dx = fmaxf(ahi.x, bhi.x) - fminf(alo.x, blo.x);
    const float dy = fmaxf(ahi.y, bhi.y) - fminf(alo.y, blo.y);
    const float dz = fmaxf(ahi.z, bhi.z) - fminf(alo.z, blo.z);
    return dx * dy + dy * dz + dz * dx;
}

// Leaf clusters in Morton order + the leaf-order triangle packs (refit's K5).
__global__ __launch_bounds__(kBlock) void k_ploc_init(int n, const uint32_t* __restrict__ order,
                                                      const float4* __restrict__ world,
                                                      const int32_t* __restrict__ tri_mat,
                                                      float4* __restrict__ cl, TriPack* __restrict__ tris) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int orig = (int)order[i];
    const float4 a = world[3 * orig], b = world[3 * orig + 1], c = world[3 * orig + 2];
    TriPack tp;
    tp.p0 = make_float4(a.x, a.y, a.z, i2f(orig));
    tp.p1 = make_float4(b.x, b.y, b.z, i2f(tri_mat[orig]));
    tp.p2 = make_float4(c.x, c.y, c.z, 0.0f);
    tris[i] = tp;
    cl[2 * i] = make_float4(fminf(fminf(a.x, b.x), c.x), fminf(fminf(a.y, b.y), c.y), fminf(fminf(a.z, b.z), c.z),
                            i2f(~i));
    cl[2 * i + 1] = make_float4(fmaxf(fmaxf(a.x, b.x), c.x), fmaxf(fmaxf(a.y, b.y), c.y),
                                fmaxf(fmaxf(a.z, b.z), c.z), 0.0f);
}

// Nearest neighbour within kPlocR positions (ascending scan, strict <).
__global__ __launch_bounds__(kBlock) void k_ploc_nn(const int* __restrict__ cnt_in, const float4* __restrict__ cl,
                                                    int* __restrict__ nn) {
    const int cnt = *cnt_in;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= cnt) return;
    const float4 alo = cl[2 * i], ahi = cl[2 * i + 1];
    float best = __builtin_huge_valf();
    int bj = -1;
    const int j0 = max(0, i - kPlocR), j1 = min(cnt - 1, i + kPlocR);
    for (int j = j0; j <= j1; ++j) {
        if (j == i) continue;
        const float a = ploc_area(alo, ahi, cl[2 * j], cl[2 * j + 1]);
        if (a < best) {
            best = a;
            bj = j;
        }
    }
    nn[i] = bj;
}

// Flags for the two scans (length bound + 1, zero beyond the live count):
// keep[i] = position i survives (not the upper half of a merge),
// mrg[i] = position i starts a merge with nn[i] > i.
__global__ __launch_bounds__(kBlock) void k_ploc_flags(const int* __restrict__ cnt_in, int bound,
                                                       const int* __restrict__ nn, uint32_t* __restrict__ keep,
                                                       uint32_t* __restrict__ mrg) {
    const int cnt = *cnt_in;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i > bound) return;
    uint32_t k = 0, m = 0;
    if (i < cnt) {
        const int j = nn[i];
        const bool mutual = j >= 0 && nn[j] == i;
        m = (mutual && i < j) ? 1u : 0u;
        k = (mutual && j < i) ? 0u : 1u;
    }
    keep[i] = k;
    mrg[i] = m;
}

// Merge and compact (keep / mrg hold exclusive prefix sums, [bound] = totals).
__global__ __launch_bounds__(kBlock) void k_ploc_apply(const int* __restrict__ cnt_in, const int* __restrict__ next_in,
                                                       int* __restrict__ cnt_out, int* __restrict__ next_out,
                                                       int bound, const int* __restrict__ nn,
                                                       const uint32_t* __restrict__ keep,
                                                       const uint32_t* __restrict__ mrg,
                                                       const float4* __restrict__ cl, float4* __restrict__ cl_out,
                                                       BvhNode* __restrict__ nodes) {
    const int cnt = *cnt_in, next = *next_in;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) {
        *cnt_out = (int)keep[bound];
        *next_out = next - (int)mrg[bound];
    }
    if (i >= cnt) return;
    const int j = nn[i];
    const bool mutual = j >= 0 && nn[j] == i;
    if (mutual && j < i) return;  // merged into position j
    const float4 alo = cl[2 * i], ahi = cl[2 * i + 1];
    const uint32_t o = keep[i];
    if (mutual) {
        const int idx = next - (int)mrg[i];
        const float4 blo = cl[2 * j], bhi = cl[2 * j + 1];
        BvhNode nd;
        nd.a = make_float4(alo.x, alo.y, alo.z, ahi.x);
        nd.b = make_float4(ahi.y, ahi.z, blo.x, blo.y);
        nd.c = make_float4(blo.z, bhi.x, bhi.y, bhi.z);
        nd.d = make_int4(f2i(alo.w), f2i(blo.w), 0, 0);  // child refs
        nodes[idx] = nd;
        cl_out[2 * o] = make_float4(fminf(alo.x, blo.x), fminf(alo.y, blo.y), fminf(alo.z, blo.z), i2f(idx));
        cl_out[2 * o + 1] = make_float4(fmaxf(ahi.x, bhi.x), fmaxf(ahi.y, bhi.y), fmaxf(ahi.z, bhi.z), 0.0f);
    } else {
        cl_out[2 * o] = alo;
        cl_out[2 * o + 1] = ahi;
    }
}

// ------------------------------------------------------- one-launch build ---
// Scenes of at most kSmallBuild triangles (every LDS-resident scene: 04vs and
// 01 are 12) build their whole LBVH in ONE workgroup, one thread per triangle,
// with the intermediate arrays in LDS: the multi-kernel build above is ~26
// launches (~0.14 ms of launch latency per frame at 12 triangles) around a few
// hundred instructions of work. Same results, bit for bit:
//  - K1/K2: the same float ops in the same order as k_transform / k_morton;
//  - K3: the stable LSD radix sort of (key, index = i) is the order by
//    (key, i); here each thread takes its rank by counting;
//  - K4: k_karras on the sorted keys in LDS;
//  - refit: a child's box is the min/max of the leaf boxes of its sorted leaf
//    range (min/max are exact, so any grouping gives the tree-merge values);
//  - K5 triangle packs as above.
constexpr int kSmallBuild = 512;

__global__ __launch_bounds__(kSmallBuild) void k_build_small(
    int n, const float4* __restrict__ local, const int32_t* __restrict__ obj, const float* __restrict__ xform,
    const int32_t* __restrict__ tri_mat, float4* __restrict__ world, uint32_t* __restrict__ bounds,
    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, int2* __restrict__ children,
    int32_t* __restrict__ node_parent, int32_t* __restrict__ leaf_parent, int2* __restrict__ range,
    BvhNode* __restrict__ nodes, TriPack* __restrict__ tris) {
    __shared__ uint32_t red[6];
    __shared__ uint32_t key_in[kSmallBuild], key_s[kSmallBuild];
    __shared__ float3 wv[kSmallBuild][3];  // world vertices, original order
    __shared__ float lbox[kSmallBuild][6];  // leaf boxes, sorted order
    __shared__ int2 rng[kSmallBuild];       // (first, count) per internal node
    const int i = threadIdx.x;
    if (i < 6) red[i] = i < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    float3 c = mk3(0.0f, 0.0f, 0.0f);
    if (i < n) {  // K1 (k_transform)
        const float* m = xform + 12 * obj[i];
        float3 w[3];
        for (int k = 0; k < 3; ++k) {
            const float4 v = local[3 * i + k];
            w[k] = mk3(xf(m, v.x, v.y, v.z), xf(m + 4, v.x, v.y, v.z), xf(m + 8, v.x, v.y, v.z));
            wv[i][k] = w[k];
        }
        c = add3(add3(w[0], w[1]), w[2]);
        world[3 * i + 0] = make_float4(w[0].x, w[0].y, w[0].z, c.x);
        world[3 * i + 1] = make_float4(w[1].x, w[1].y, w[1].z, c.y);
        world[3 * i + 2] = make_float4(w[2].x, w[2].y, w[2].z, c.z);
        atomicMin(&red[0], f2o(c.x));
        atomicMin(&red[1], f2o(c.y));
        atomicMin(&red[2], f2o(c.z));
        atomicMax(&red[3], f2o(c.x));
        atomicMax(&red[4], f2o(c.y));
        atomicMax(&red[5], f2o(c.z));
    }
    __syncthreads();
    if (i < 6) bounds[i] = red[i];
    if (i < n) {  // K2 (k_morton)
        const float lo[3] = {o2f(red[0]), o2f(red[1]), o2f(red[2])};
        const float hi[3] = {o2f(red[3]), o2f(red[4]), o2f(red[5])};
        const float cc[3] = {c.x, c.y, c.z};
        uint32_t q[3];
        for (int k = 0; k < 3; ++k) {
            const float ext = hi[k] - lo[k];
            const float s = ext > 0.0f ? 1024.0f / ext : 0.0f;
            float f = (cc[k] - lo[k]) * s;
            f = fminf(fmaxf(f, 0.0f), 1023.0f);
            q[k] = (uint32_t)f;
        }
        key_in[i] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    }
    __syncthreads();
    if (i < n) {  // K3: rank of (key, i)
        const uint32_t k = key_in[i];
        int r = 0;
        for (int j = 0; j < n; ++j) {
            const uint32_t kj = key_in[j];
            r += (kj < k || (kj == k && j < i)) ? 1 : 0;
        }
        key_s[r] = k;
        keys[r] = k;
        vals[r] = (uint32_t)i;
        // K5 pack of sorted leaf r (k_refit) and its box
        const float3 a = wv[i][0], b = wv[i][1], e = wv[i][2];
        TriPack tp;
        tp.p0 = make_float4(a.x, a.y, a.z, i2f(i));
        tp.p1 = make_float4(b.x, b.y, b.z, i2f(tri_mat[i]));
        tp.p2 = make_float4(e.x, e.y, e.z, 0.0f);
        tris[r] = tp;
        lbox[r][0] = fminf(fminf(a.x, b.x), e.x);
        lbox[r][1] = fminf(fminf(a.y, b.y), e.y);
        lbox[r][2] = fminf(fminf(a.z, b.z), e.z);
        lbox[r][3] = fmaxf(fmaxf(a.x, b.x), e.x);
        lbox[r][4] = fmaxf(fmaxf(a.y, b.y), e.y);
        lbox[r][5] = fmaxf(fmaxf(a.z, b.z), e.z);
    }
    __syncthreads();
    if (n == 1) {  // single triangle: root with both children = leaf 0 (k_refit)
        if (i == 0) {
            float* f = reinterpret_cast<float*>(&nodes[0]);
            for (int k = 0; k < 6; ++k) {
                f[k] = lbox[0][k];
                f[6 + k] = lbox[0][k];
            }
            nodes[0].d = make_int4(~0, ~0, 0, 0);
        }
        return;
    }
    int2 ch = make_int2(0, 0);
    if (i < n - 1) {  // K4a (k_karras) over the sorted keys in LDS
        const int d = (delta(key_s, n, i, i + 1) - delta(key_s, n, i, i - 1)) >= 0 ? 1 : -1;
        const int dmin = delta(key_s, n, i, i - d);
        int lmax = 2;
        while (delta(key_s, n, i, i + lmax * d) > dmin) lmax <<= 1;
        int l = 0;
        for (int t = lmax >> 1; t >= 1; t >>= 1)
            if (delta(key_s, n, i, i + (l + t) * d) > dmin) l += t;
        const int j = i + l * d;
        const int dnode = delta(key_s, n, i, j);
        int s = 0;
        int t = l;
        do {
            t = (t + 1) >> 1;
            if (delta(key_s, n, i, i + (s + t) * d) > dnode) s += t;
        } while (t > 1);
        const int gamma = i + s * d + (d < 0 ? -1 : 0);
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        if (lo == gamma) {
            ch.x = ~gamma;
            leaf_parent[gamma] = 2 * i;
        } else {
            ch.x = gamma;
            node_parent[gamma] = 2 * i;
        }
        if (hi == gamma + 1) {
            ch.y = ~(gamma + 1);
            leaf_parent[gamma + 1] = 2 * i + 1;
        } else {
            ch.y = gamma + 1;
            node_parent[gamma + 1] = 2 * i + 1;
        }
        children[i] = ch;
        rng[i] = make_int2(lo, hi - lo + 1);
        range[i] = rng[i];
        if (i == 0) node_parent[0] = -1;
    }
    __syncthreads();
    if (i < n - 1) {  // K4b refit from leaf ranges
        float f[12];
        int ref[2] = {ch.x, ch.y};
        for (int side = 0; side < 2; ++side) {
            const int cref = side ? ch.y : ch.x;
            int first, cnt;
            if (cref < 0) {
                first = ~cref;
                cnt = 1;
            } else {
                first = rng[cref].x;
                cnt = rng[cref].y;
            }
            float bx[6];
            for (int k = 0; k < 6; ++k) bx[k] = lbox[first][k];
            for (int q = first + 1; q < first + cnt; ++q) {
                for (int k = 0; k < 3; ++k) bx[k] = fminf(bx[k], lbox[q][k]);
                for (int k = 3; k < 6; ++k) bx[k] = fmaxf(bx[k], lbox[q][k]);
            }
            for (int k = 0; k < 6; ++k) f[6 * side + k] = bx[k];
        }
        BvhNode nd;
        nd.a = make_float4(f[0], f[1], f[2], f[3]);
        nd.b = make_float4(f[4], f[5], f[6], f[7]);
        nd.c = make_float4(f[8], f[9], f[10], f[11]);
        nd.d = make_int4(ref[0], ref[1], 0, 0);
        nodes[i] = nd;
    }
}

struct UploadArgs {
    float* dst[3];
    int n[3];
    float data[kUploadMax];
};

__global__ __launch_bounds__(kBlock) void k_upload(UploadArgs a) {
    int off = 0;
    for (int k = 0; k < 3; ++k) {
        for (int i = threadIdx.x; i < a.n[k]; i += kBlock) a.dst[k][i] = a.data[off + i];
        off += a.n[k];
    }
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

void exclusive_scan(DevScene& s, uint32_t* data, int m, hipStream_t st) {
    const int tiles = cdiv(m, kScanTile);
    s.scan_part.ensure((size_t)tiles);
    k_scan_tiles<<<tiles, kBlock, 0, st>>>(m, data, s.scan_part.ptr);
    k_scan_parts<<<1, kBlock, 0, st>>>(tiles, s.scan_part.ptr);
    k_scan_add<<<tiles, kBlock, 0, st>>>(m, data, s.scan_part.ptr);
}

}  // namespace

bool upload_by_kernarg(const float* src, const UploadSeg* segs, int nseg, hipStream_t st) {
    if (nseg > 3) return false;
    UploadArgs a{};
    int total = 0;
    for (int k = 0; k < nseg; ++k) total += segs[k].n;
    if (total > kUploadMax) return false;
    for (int k = 0; k < nseg; ++k) {
        a.dst[k] = segs[k].dst;
        a.n[k] = segs[k].n;
    }
    std::memcpy(a.data, src, total * sizeof(float));
    k_upload<<<1, kBlock, 0, st>>>(a);
    RR_HIP(hipGetLastError());
    return true;
}

void DevScene::release() {
    tri_local.release(); tri_obj.release(); tri_mat.release(); obj_xform.release();
    tri_world.release(); bounds.release();
    for (int k = 0; k < 2; ++k) { keys[k].release(); vals[k].release(); }
    hist.release(); scan_part.release(); children.release(); node_parent.release();
    leaf_parent.release(); flags.release(); nodes.release(); tris.release(); qnodes.release(); qtris.release(); q_src.release(); q_cnt.release(); q_tcnt.release(); q_ctl.release();
    range.release();
    tnrm.release();
    for (int k = 0; k < 2; ++k) ploc_cl[k].release();
    ploc_nn.release(); ploc_keep.release(); ploc_mrg.release(); ploc_ctl.release();
    has4 = false;
    ploc = false;
    built = false;
    uploaded = false;
}

// PLOC rounds after the Morton sort (sorted order in vals[0]).
void build_ploc(DevScene& s, hipStream_t st) {
    const int n = s.n_tris;
    s.ploc_cl[0].ensure((size_t)2 * n);
    s.ploc_cl[1].ensure((size_t)2 * n);
    s.ploc_nn.ensure((size_t)n);
    s.ploc_keep.ensure((size_t)n + 1);
    s.ploc_mrg.ensure((size_t)n + 1);
    s.ploc_ctl.ensure(4);
    k_ploc_init<<<cdiv(n, kBlock), kBlock, 0, st>>>(n, s.vals[0].ptr, s.tri_world.ptr, s.tri_mat.ptr,
                                                     s.ploc_cl[0].ptr, s.tris.ptr);
    const int init[4] = {n, n - 2, 0, 0};  // ctl[0/1]: count ping-pong, ctl[2/3]: next-index ping-pong
    const int ctl_host[4] = {init[0], 0, init[1], 0};
    RR_HIP(hipMemcpyAsync(s.ploc_ctl.ptr, ctl_host, sizeof ctl_host, hipMemcpyHostToDevice, st));
    RR_HIP(hipStreamSynchronize(st));  // ctl_host is on the stack
    int bound = n, cur = 0, rounds = 0;
    for (;;) {
        // a batch of rounds without host synchronisation; kernels read the live count
        for (int r = 0; r < 4; ++r, ++rounds) {
            int* cin = s.ploc_ctl.ptr + cur;
            int* cout = s.ploc_ctl.ptr + (1 - cur);
            int* nin = s.ploc_ctl.ptr + 2 + cur;
            int* nout = s.ploc_ctl.ptr + 2 + (1 - cur);
            const int g = cdiv(bound + 1, kBlock);
            k_ploc_nn<<<g, kBlock, 0, st>>>(cin, s.ploc_cl[cur].ptr, s.ploc_nn.ptr);
            k_ploc_flags<<<g, kBlock, 0, st>>>(cin, bound, s.ploc_nn.ptr, s.ploc_keep.ptr, s.ploc_mrg.ptr);
            exclusive_scan(s, s.ploc_keep.ptr, bound + 1, st);
            exclusive_scan(s, s.ploc_mrg.ptr, bound + 1, st);
            k_ploc_apply<<<g, kBlock, 0, st>>>(cin, nin, cout, nout, bound, s.ploc_nn.ptr, s.ploc_keep.ptr,
                                               s.ploc_mrg.ptr, s.ploc_cl[cur].ptr, s.ploc_cl[1 - cur].ptr,
                                               s.nodes.ptr);
            cur = 1 - cur;
        }
        int cnt = 0;
        RR_HIP(hipMemcpyAsync(&cnt, s.ploc_ctl.ptr + cur, sizeof cnt, hipMemcpyDeviceToHost, st));
        RR_HIP(hipStreamSynchronize(st));
        if (cnt <= 1) break;
        if (cnt >= bound || rounds > 4 * 64 + 2 * n) throw std::runtime_error("PLOC made no progress");
        bound = cnt;
    }
}

// The shading terms of each triangle of the split path, in leaf order: the
// unit geometric normal (the same norm3(cross3(e1, e2)) shade() computes
// from the triangle record, contraction off: the same bits) and the material
// id, one 16 B read per shading point instead of the 48 B record and a cross
// product (wavefront.hip shade(), RR_SHADE_NRM).
__global__ __launch_bounds__(kBlock) void k_tri_nrm(const TriPack* __restrict__ tris, int n, float4* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const TriPack tp = tris[i];
    const float3 N = norm3(cross3(sub3(xyz(tp.p1), xyz(tp.p0)), sub3(xyz(tp.p2), xyz(tp.p0))));
    out[i] = make_float4(N.x, N.y, N.z, tp.p1.w);
}

// Quantised 6-wide hierarchy of the built BVH2 (kernels above): one count / scan / emit /
// advance round per level; the host learns the frontier size every 4 levels
// (one synchronisation) and sizes the next launches by it (a level has at
// most kQWidth x the nodes of the one before).
void build_qbvh(DevScene& s, hipStream_t st) {
    const int n = s.n_tris;
    const int ni = n > 1 ? n - 1 : 1;
    // the walks' grouped stack entries hold a node index in 26 bits (rr_device.h pop_group)
    if (ni >= (1 << 26)) throw std::runtime_error("scene too large for the 6-wide hierarchy (2^26 nodes)");
    s.qnodes.ensure((size_t)ni);
    s.qtris.ensure((size_t)n);
    s.q_src.ensure((size_t)ni);
    s.q_cnt.ensure((size_t)ni + 1);
    s.q_tcnt.ensure((size_t)ni + 1);
    s.q_ctl.ensure(3);
    k_qw_init<<<1, 1, 0, st>>>(s.q_ctl.ptr, s.q_src.ptr);
    long frontier = 1;  // bound on the current level's node count
    for (int level = 0;; ++level) {
        const int bound = (int)std::min<long>(frontier, ni);
        k_qw_count<<<cdiv(bound + 1, kBlock), kBlock, 0, st>>>(s.q_ctl.ptr, bound, n, s.nodes.ptr, s.q_src.ptr,
                                                                s.q_cnt.ptr, s.q_tcnt.ptr);
        exclusive_scan(s, s.q_cnt.ptr, bound + 1, st);
        exclusive_scan(s, s.q_tcnt.ptr, bound + 1, st);
        k_qw_emit<<<cdiv(bound, kBlock), kBlock, 0, st>>>(s.q_ctl.ptr, bound, n, s.nodes.ptr, s.q_src.ptr,
                                                           s.q_cnt.ptr, s.q_tcnt.ptr, s.tris.ptr, s.qtris.ptr,
                                                           s.qnodes.ptr);
        k_qw_advance<<<1, 1, 0, st>>>(s.q_ctl.ptr, bound, s.q_cnt.ptr, s.q_tcnt.ptr);
        frontier = std::min<long>(frontier * kQWidth, ni);  // a level has at most kQWidth x the nodes of the one before
        if ((level & 3) == 3) {
            int ctl[2];
            RR_HIP(hipMemcpyAsync(ctl, s.q_ctl.ptr, sizeof ctl, hipMemcpyDeviceToHost, st));
            RR_HIP(hipStreamSynchronize(st));
            if (ctl[0] == ctl[1]) {
                s.nq = ctl[1];
                break;
            }
            frontier = ctl[1] - ctl[0];
            if (level > 4 * 4096) throw std::runtime_error("6-wide collapse made no progress");
        }
    }
    std::swap(s.tris, s.qtris);  // the traversal and shading read the 6-wide hierarchy's leaf order
    s.tnrm.ensure((size_t)std::max(n, 1));
    if (n > 0) k_tri_nrm<<<cdiv(n, kBlock), kBlock, 0, st>>>(s.tris.ptr, n, s.tnrm.ptr);
    s.has4 = true;
}

void build_lbvh(DevScene& s, hipStream_t st, KernelProfiler* prof, bool want4, bool want_ploc) {
    const int n = s.n_tris;
    s.has4 = false;
    if (n <= 0) {
        s.built = true;
        return;
    }
    if (prof) prof->begin(st, 0);
    const int nb = cdiv(n, kBlock);
    s.tri_world.ensure((size_t)3 * n);
    s.bounds.ensure(6);
    for (int k = 0; k < 2; ++k) {
        s.keys[k].ensure((size_t)n);
        s.vals[k].ensure((size_t)n);
    }
    s.nodes.ensure((size_t)(n > 1 ? n - 1 : 1));
    s.tris.ensure((size_t)n);
    s.children.ensure((size_t)(n > 1 ? n - 1 : 1));
    s.node_parent.ensure((size_t)(n > 1 ? n - 1 : 1));
    s.leaf_parent.ensure((size_t)n);
    s.flags.ensure((size_t)(n > 1 ? n - 1 : 1));
    s.range.ensure((size_t)(n > 1 ? n - 1 : 1));

    if (n <= kSmallBuild && !want4 && !(want_ploc && n > 2)) {
        k_build_small<<<1, kSmallBuild, 0, st>>>(n, s.tri_local.ptr, s.tri_obj.ptr, s.obj_xform.ptr, s.tri_mat.ptr,
                                                 s.tri_world.ptr, s.bounds.ptr, s.keys[0].ptr, s.vals[0].ptr,
                                                 s.children.ptr, s.node_parent.ptr, s.leaf_parent.ptr, s.range.ptr,
                                                 s.nodes.ptr, s.tris.ptr);
        if (prof) prof->end(st);
        RR_HIP(hipGetLastError());
        s.ploc = false;
        s.built = true;
        return;
    }

    RR_HIP(hipMemsetAsync(s.bounds.ptr, 0xFF, 3 * sizeof(uint32_t), st));
    RR_HIP(hipMemsetAsync(s.bounds.ptr + 3, 0x00, 3 * sizeof(uint32_t), st));
    k_transform<<<nb, kBlock, 0, st>>>(n, s.tri_local.ptr, s.tri_obj.ptr, s.obj_xform.ptr,
                                        s.tri_world.ptr, s.bounds.ptr);
    k_morton<<<nb, kBlock, 0, st>>>(n, s.tri_world.ptr, s.bounds.ptr, s.keys[0].ptr, s.vals[0].ptr);
    // K3: four stable 8-bit passes over the 30-bit keys
    const int sb = cdiv(n, kSortTile);
    const int m = 256 * sb;
    s.hist.ensure((size_t)m);
    int cur = 0;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 8 * pass;
        k_radix_hist<<<sb, kBlock, 0, st>>>(n, shift, s.keys[cur].ptr, s.hist.ptr, sb);
        exclusive_scan(s, s.hist.ptr, m, st);
        k_radix_scatter<<<sb, kBlock, 0, st>>>(n, shift, s.keys[cur].ptr, s.vals[cur].ptr,
                                               s.keys[1 - cur].ptr, s.vals[1 - cur].ptr, s.hist.ptr, sb);
        cur = 1 - cur;
    }
    if (cur != 0) {  // keep sorted data in slot 0 (4 passes: already back in 0)
        std::swap(s.keys[0], s.keys[1]);
        std::swap(s.vals[0], s.vals[1]);
    }
    s.ploc = want_ploc && n > 2;
    if (s.ploc) {
        build_ploc(s, st);
    } else if (n > 1) {
        k_karras<<<cdiv(n - 1, kBlock), kBlock, 0, st>>>(n, s.keys[0].ptr, s.children.ptr,
                                                          s.node_parent.ptr, s.leaf_parent.ptr, s.range.ptr);
        RR_HIP(hipMemsetAsync(s.flags.ptr, 0, (size_t)(n - 1) * sizeof(uint32_t), st));
    }
    if (!s.ploc)
        k_refit<<<nb, kBlock, 0, st>>>(n, s.vals[0].ptr, s.tri_world.ptr, s.tri_mat.ptr, s.leaf_parent.ptr,
                                       s.node_parent.ptr, s.children.ptr, s.flags.ptr, s.nodes.ptr,
                                       s.tris.ptr);
    if (want4) build_qbvh(s, st);
    if (prof) prof->end(st);
    RR_HIP(hipGetLastError());
    s.built = true;
}

}  // namespace rr
