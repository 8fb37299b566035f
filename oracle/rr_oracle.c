/*
 * rr_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the renderer's
 * hot path, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker. The product (librr.so) never links or calls
 * this file.
 *
 * What it restates, and from where:
 *  - The reference's per-frame render step is Blender 3.6.0 Cycles on the CPU
 *    (/root/reference/worker/src/rendering/runner/mod.rs:165-174 spawns
 *    `blender`; /root/reference/scripts/render-timing-script.py:90 calls
 *    bpy.ops.render.render). Cycles is a third-party dependency absent from
 *    /root/reference (pinned only as the docker image linuxserver/blender:3.6.0,
 *    /root/reference/pull-blender-image.sh:3-4), so Cycles-image parity is
 *    UNPINNED here; see DESIGN.md §5.
 *  - This oracle is the specification of the MI355X renderer's algorithm
 *    (DESIGN.md §4): Karras LBVH over 30-bit Morton codes (PLOC over the same
 *    sorted leaves for scenes traversed from HBM), closest/any-hit
 *    traversal with an order-independent accept rule, a path tracer with the
 *    Principled-BSDF subset, point/sun NEE, Cycles-style light units
 *    (point: P/(4 pi) W/sr, eval_fac 1/(4 pi) * invarea), indirect clamp,
 *    Russian roulette, Blackman-Harris filter importance sampling, sRGB
 *    "Standard" view transform and 8-bit quantisation as Blender's
 *    unit_float_to_uchar_clamp.
 *  - Written scalar, one path at a time, in the same IEEE single-precision
 *    operation order as the HIP kernels, without contraction (built with
 *    -ffp-contract=off): a fused multiply-add happens exactly where both
 *    sides spell fmaf() (C99 fmaf is correctly rounded, as v_fma_f32 is; -mfma
 *    makes it one instruction), and without libm transcendentals on the
 *    per-sample path, so GPU and oracle agree bit for bit on identical inputs
 *    (tests/test_gpu_parity.py).
 *  - Pinning of this oracle against analytic known answers (white furnace,
 *    point-light closed form, ray/triangle and LBVH vs brute force):
 *    tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_FILTER_N 1024
#define ORC_SRGB_N 4096
#define ORC_SEG 64       /* pixels per OpenMP work item of orc_render */
#define ORC_MAXDEPTH 80 /* = the GPU traversal stack (kLdsStack + kSpillStack, rr_device.h) */

typedef struct { float x, y, z; } v3;

static v3 V(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static v3 vscl(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
/* products accumulate through fmaf (rr_device.h dot3 / cross3 / madd3 / frame3) */
static float vdot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static v3 vcross(v3 a, v3 b) {
    return V(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static v3 vmadd(v3 a, v3 b, float s) { return V(fmaf(b.x, s, a.x), fmaf(b.y, s, a.y), fmaf(b.z, s, a.z)); }
static v3 vframe(v3 t, v3 u, v3 w, float x, float y, float z) {
    return V(fmaf(w.x, z, fmaf(u.x, y, t.x * x)), fmaf(w.y, z, fmaf(u.y, y, t.y * x)), fmaf(w.z, z, fmaf(u.z, y, t.z * x)));
}
static v3 vnorm(v3 a) { float inv = 1.0f / sqrtf(vdot(a, a)); return vscl(a, inv); }
static float vmax3(v3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }

static int fbits(float f) { int i; memcpy(&i, &f, 4); return i; }
static float ibits(int i) { float f; memcpy(&f, &i, 4); return f; }

/* ------------------------------------------------------------ tables ---- */
/* Blackman-Harris inverse-CDF table, support [-w, w] (Cycles doubles the BH
 * filter width). Double precision, midpoint rule on 16*N cells. */
void orc_filter_table(float width, float* table) {
    const int N = ORC_FILTER_N, M = 16 * ORC_FILTER_N;
    const double w = 2.0 * (double)width;
    double* cdf = (double*)calloc((size_t)M + 1, sizeof(double));
    for (int i = 0; i < M; ++i) {
        double x = ((double)i + 0.5) / M;
        double v = 2.0 * M_PI * x;
        double f = 0.35875 - 0.48829 * cos(v) + 0.14128 * cos(2.0 * v) - 0.01168 * cos(3.0 * v);
        cdf[i + 1] = cdf[i] + (f > 0.0 ? f : 0.0);
    }
    for (int i = 0; i <= M; ++i) cdf[i] /= cdf[M];
    int j = 0;
    for (int i = 0; i < N; ++i) {
        double u = (double)i / (N - 1);
        while (j < M - 1 && cdf[j + 1] < u) ++j;
        double d = cdf[j + 1] - cdf[j];
        double fr = d > 0.0 ? (u - cdf[j]) / d : 0.0;
        if (fr < 0.0) fr = 0.0;
        if (fr > 1.0) fr = 1.0;
        double x = ((double)j + fr) / M;
        table[i] = (float)(w * (x - 0.5));
    }
    free(cdf);
}

void orc_srgb_lut(float* lut) {
    for (int i = 0; i <= ORC_SRGB_N; ++i) lut[i] = (float)(1.055 * pow((double)i / ORC_SRGB_N, 1.0 / 2.4) - 0.055);
}

static float lerp_table(const float* t, int n, float u) {
    float f = u * (float)(n - 1);
    int i = (int)f;
    if (i >= n - 1) return t[n - 1];
    if (i < 0) i = 0;
    float fr = f - (float)i;
    return fmaf(t[i + 1] - t[i], fr, t[i]);
}

/* --------------------------------------------------------------- RNG ---- */
static uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
static uint32_t pkey(uint32_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t k = hash32(hash32(seed) + pixel);
    return hash32(k ^ (sample * 0x9E3779B9u + 0x7F4A7C15u));
}
static float rnd(uint32_t key, uint32_t dim) {
    return (float)(hash32(key + (dim + 1u) * 0x9E3779B9u) >> 8) * 5.9604644775390625e-08f;
}
/* two uniforms of one hash, 16 bits each (csrc/rr_device.h rng2): the
 * dimension pairs of a sample (camera subpixel, light pick + lobe choice,
 * disk point, BSDF direction) */
static void rnd2(uint32_t key, uint32_t dim, float* a, float* b) {
    const uint32_t h = hash32(key + (dim + 1u) * 0x9E3779B9u);
    *a = (float)(h >> 16) * 1.52587890625e-05f;
    *b = (float)(h & 0xffffu) * 1.52587890625e-05f;
}

/* ---------------------------------------------------------- sampling ---- */
static void small_sincos(float x, float* s, float* c) {
    float z = x * x;
    float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    *s = fmaf(ps * z, x, x);
    float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    *c = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
}

static void disk(float u1, float u2, float* x, float* y) {
    float a = fmaf(2.0f, u1, -1.0f), b = fmaf(2.0f, u2, -1.0f), s, c;
    if (a == 0.0f && b == 0.0f) { *x = 0.0f; *y = 0.0f; return; }
    if (fabsf(a) > fabsf(b)) {
        small_sincos(0.785398163397448f * (b / a), &s, &c);
        *x = a * c; *y = a * s;
    } else {
        small_sincos(0.785398163397448f * (a / b), &s, &c);
        *x = b * s; *y = b * c;
    }
}

static void onb(v3 n, v3* b1, v3* b2) {
    float sign = copysignf(1.0f, n.z);
    float a = -1.0f / (sign + n.z);
    float b = n.x * n.y * a;
    *b1 = V(fmaf(sign * n.x * n.x, a, 1.0f), sign * b, -sign * n.x);
    *b2 = V(b, fmaf(n.y * n.y, a, sign), -n.y);
}

static float off_axis(float p, float n) {
    int of = (int)(256.0f * n);
    float pi = ibits(fbits(p) + ((p < 0.0f) ? -of : of));
    return fabsf(p) < 0.03125f ? fmaf(1.52587890625e-05f, n, p) : pi;
}
static v3 offset_ray(v3 p, v3 n) { return V(off_axis(p.x, n.x), off_axis(p.y, n.y), off_axis(p.z, n.z)); }

/* ---------------------------------------------------------------- LBVH --- */
typedef struct {
    int n;
    uint32_t* keys;   /* sorted */
    uint32_t* order;  /* sorted original ids */
    int* child;       /* 2*(n-1) or 2: full Karras topology */
    int* child_lf;    /* the same with subtrees of <= ORC_LEAF_MAX leaves as leaf ranges (what trace() walks) */
    int* range;       /* 2 per internal node: first sorted leaf, leaf count */
    float* box;       /* 12 per internal node */
    float* tri;       /* leaf order: v0 v1 v2 (9; rr_device.h TriPack) */
    int* tri_orig;
    int* tri_mat;
    int width;        /* hierarchy trace() walks: 2 (BVH2) or 4 (the quantised wide collapse, ORC_QW children) */
    int n4;           /* quantised wide nodes */
    int* child4;      /* ORC_QW per node (derived from the node, for tests): >= 0 node, < 0 ~leaf, ORC_EMPTY4 unused */
    uint32_t* q4;     /* 16 words per node, csrc/rr_device.h QNode6 */
} lbvh;

#define ORC_EMPTY4 0x7fffffff
/* Leaf refs name ranges of sorted leaves, ~(first | (count-1) << 28), for
 * subtrees of at most ORC_LEAF_MAX leaves (rr_device.h kLeafMax, bvh.hip
 * k_leafify; the two constants must be equal). */
#define ORC_LEAF_MAX 1
static int leaf_ref(int first, int count) { return ~(first | ((count - 1) << 28)); }
static int leaf_first(int ref) { return (~ref) & 0x0FFFFFFF; }
static int leaf_count(int ref) { return ((~ref) >> 28) + 1; }

static uint32_t spread10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

static int clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }

static int kdelta(const uint32_t* k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    if (k[i] == k[j]) return 32 + clz32((uint32_t)(i ^ j));
    return clz32(k[i] ^ k[j]);
}

static void tri_box(const float* t9, float b[6]) {
    for (int a = 0; a < 3; ++a) {
        b[a] = fminf(fminf(t9[a], t9[3 + a]), t9[6 + a]);
        b[3 + a] = fmaxf(fmaxf(t9[a], t9[3 + a]), t9[6 + a]);
    }
}

/* box of the subtree rooted at child code c */
static void subtree_box(const lbvh* B, const float* tris9, int c, float out[6]) {
    if (c < 0) {
        tri_box(tris9 + 9 * (size_t)B->order[~c], out);
        return;
    }
    const float* bx = B->box + 12 * (size_t)c;
    for (int a = 0; a < 3; ++a) {
        out[a] = fminf(bx[a], bx[6 + a]);
        out[3 + a] = fmaxf(bx[3 + a], bx[9 + a]);
    }
}

static void lbvh_free(lbvh* B) {
    free(B->child4); free(B->q4); free(B->child_lf); free(B->range);
    free(B->keys); free(B->order); free(B->child); free(B->box);
    free(B->tri); free(B->tri_orig); free(B->tri_mat);
    memset(B, 0, sizeof *B);
}

static void ploc_build(lbvh* B, const float* tris9);

/* hier: 2 = Karras LBVH, 3 = PLOC over the same sorted leaves (csrc/bvh.hip
 * build_ploc), 4 = LBVH (collapsed to the BVH4 by the caller). */
static void lbvh_build(lbvh* B, int n, const float* tris9, const int* mats, int hier) {
    memset(B, 0, sizeof *B);
    B->n = n;
    if (n <= 0) return;
    B->keys = (uint32_t*)malloc(sizeof(uint32_t) * n);
    B->order = (uint32_t*)malloc(sizeof(uint32_t) * n);
    float* cen = (float*)malloc(sizeof(float) * 3 * (size_t)n);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n; ++i) {
        const float* t = tris9 + 9 * (size_t)i;
        for (int a = 0; a < 3; ++a) {
            float c = (t[a] + t[3 + a]) + t[6 + a];  /* centroid sum */
            cen[3 * (size_t)i + a] = c;
            if (c < lo[a]) lo[a] = c;
            if (c > hi[a]) hi[a] = c;
        }
    }
    uint32_t* tmpk = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* tmpv = (uint32_t*)malloc(sizeof(uint32_t) * n);
    for (int i = 0; i < n; ++i) {
        uint32_t q[3];
        for (int a = 0; a < 3; ++a) {
            float ext = hi[a] - lo[a];
            float s = ext > 0.0f ? 1024.0f / ext : 0.0f;
            float f = (cen[3 * (size_t)i + a] - lo[a]) * s;
            f = fminf(fmaxf(f, 0.0f), 1023.0f);
            q[a] = (uint32_t)f;
        }
        tmpk[i] = (spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]);
        tmpv[i] = (uint32_t)i;
    }
    /* stable counting sort, 4 x 8 bits (LSD) */
    for (int pass = 0; pass < 4; ++pass) {
        int shift = 8 * pass;
        size_t cnt[257] = {0};
        for (int i = 0; i < n; ++i) cnt[((tmpk[i] >> shift) & 255u) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (int i = 0; i < n; ++i) {
            uint32_t d = (tmpk[i] >> shift) & 255u;
            size_t pos = cnt[d]++;
            B->keys[pos] = tmpk[i];
            B->order[pos] = tmpv[i];
        }
        memcpy(tmpk, B->keys, sizeof(uint32_t) * n);
        memcpy(tmpv, B->order, sizeof(uint32_t) * n);
    }
    free(tmpk); free(tmpv); free(cen);
    int ni = n > 1 ? n - 1 : 1;
    B->child = (int*)malloc(sizeof(int) * 2 * (size_t)ni);
    B->child_lf = (int*)malloc(sizeof(int) * 2 * (size_t)ni);
    B->range = (int*)malloc(sizeof(int) * 2 * (size_t)ni);
    B->box = (float*)malloc(sizeof(float) * 12 * (size_t)ni);
    if (hier == 3 && n > 2) {
        ploc_build(B, tris9);
        for (int i = 0; i < 2 * ni; ++i) { B->child_lf[i] = B->child[i]; B->range[i] = 0; }
        goto pack;
    }
    if (n == 1) {
        B->child[0] = ~0; B->child[1] = ~0;
    } else {
        const uint32_t* k = B->keys;
        for (int i = 0; i < n - 1; ++i) {
            int d = (kdelta(k, n, i, i + 1) - kdelta(k, n, i, i - 1)) >= 0 ? 1 : -1;
            int dmin = kdelta(k, n, i, i - d);
            int lmax = 2;
            while (kdelta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
            int l = 0;
            for (int t = lmax >> 1; t >= 1; t >>= 1)
                if (kdelta(k, n, i, i + (l + t) * d) > dmin) l += t;
            int j = i + l * d;
            int dn = kdelta(k, n, i, j);
            int s = 0, t = l;
            do {
                t = (t + 1) >> 1;
                if (kdelta(k, n, i, i + (s + t) * d) > dn) s += t;
            } while (t > 1);
            int g = i + s * d + (d < 0 ? -1 : 0);
            int lo_ = i < j ? i : j, hi_ = i < j ? j : i;
            B->child[2 * i] = (lo_ == g) ? ~g : g;
            B->child[2 * i + 1] = (hi_ == g + 1) ? ~(g + 1) : g + 1;
            B->range[2 * i] = lo_;
            B->range[2 * i + 1] = hi_ - lo_ + 1;
        }
    }
    /* boxes bottom-up: children of node i have larger indices or are leaves?
     * Not guaranteed for Karras; use an explicit post-order walk. */
    {
        int* stack = (int*)malloc(sizeof(int) * 2 * (size_t)ni + 16);
        unsigned char* done = (unsigned char*)calloc((size_t)ni, 1);
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            int v = stack[sp - 1];
            int c0 = B->child[2 * v], c1 = B->child[2 * v + 1];
            int ready = 1;
            if (n > 1) {
                if (c0 >= 0 && !done[c0]) { stack[sp++] = c0; ready = 0; }
                if (c1 >= 0 && !done[c1]) { stack[sp++] = c1; ready = 0; }
            }
            if (!ready) continue;
            --sp;
            float b0[6], b1[6];
            subtree_box(B, tris9, c0, b0);
            subtree_box(B, tris9, c1, b1);
            memcpy(B->box + 12 * (size_t)v, b0, sizeof b0);
            memcpy(B->box + 12 * (size_t)v + 6, b1, sizeof b1);
            done[v] = 1;
        }
        free(stack); free(done);
    }
    for (int i = 0; i < 2 * ni; ++i) {
        int c = B->child[i];
        B->child_lf[i] = (n > 1 && c >= 0 && B->range[2 * c + 1] <= ORC_LEAF_MAX)
                             ? leaf_ref(B->range[2 * c], B->range[2 * c + 1]) : c;
    }
pack:
    B->tri = (float*)malloc(sizeof(float) * 9 * (size_t)n);
    B->tri_orig = (int*)malloc(sizeof(int) * n);
    B->tri_mat = (int*)malloc(sizeof(int) * n);
    for (int i = 0; i < n; ++i) {
        const float* t = tris9 + 9 * (size_t)B->order[i];
        float* o = B->tri + 9 * (size_t)i;
        memcpy(o, t, 9 * sizeof(float));
        B->tri_orig[i] = (int)B->order[i];
        B->tri_mat[i] = mats ? mats[B->order[i]] : 0;
    }
}

/* PLOC (Meister & Bittner 2018), as csrc/bvh.hip build_ploc: clusters start as
 * the Morton-sorted leaves; each round every cluster takes the neighbour within
 * ORC_PLOC_R positions with the smallest merged-box measure dx*dy + dy*dz +
 * dz*dx (ascending scan, strict <: ties -> lower position), mutual nearest
 * neighbours merge (the lower position keeps the new cluster), survivors are
 * compacted in order; merge q of a round gets node index next - q, next
 * starts at n-2 and drops by the round's merges, so the root is node 0. */
#define ORC_PLOC_R 16
static float ploc_area(const float* a, const float* b) {
    float dx = fmaxf(a[3], b[3]) - fminf(a[0], b[0]);
    float dy = fmaxf(a[4], b[4]) - fminf(a[1], b[1]);
    float dz = fmaxf(a[5], b[5]) - fminf(a[2], b[2]);
    return dx * dy + dy * dz + dz * dx;
}

static void ploc_build(lbvh* B, const float* tris9) {
    const int n = B->n;
    int* ref = (int*)malloc(sizeof(int) * (size_t)n);
    int* ref2 = (int*)malloc(sizeof(int) * (size_t)n);
    float* box = (float*)malloc(sizeof(float) * 6 * (size_t)n);
    float* box2 = (float*)malloc(sizeof(float) * 6 * (size_t)n);
    int* nn = (int*)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        tri_box(tris9 + 9 * (size_t)B->order[i], box + 6 * (size_t)i);
        ref[i] = ~i;
    }
    int cnt = n, next = n - 2;
    while (cnt > 1) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int i = 0; i < cnt; ++i) {
            float best = INFINITY;
            int bj = -1;
            int j0 = i - ORC_PLOC_R < 0 ? 0 : i - ORC_PLOC_R;
            int j1 = i + ORC_PLOC_R > cnt - 1 ? cnt - 1 : i + ORC_PLOC_R;
            for (int j = j0; j <= j1; ++j) {
                if (j == i) continue;
                float a = ploc_area(box + 6 * (size_t)i, box + 6 * (size_t)j);
                if (a < best) { best = a; bj = j; }
            }
            nn[i] = bj;
        }
        int q = 0, k = 0;
        for (int i = 0; i < cnt; ++i) {
            int j = nn[i];
            int mutual = j >= 0 && nn[j] == i;
            if (mutual && j < i) continue;
            const float* a = box + 6 * (size_t)i;
            float* o = box2 + 6 * (size_t)k;
            if (mutual) {
                const float* b = box + 6 * (size_t)j;
                int idx = next - q++;
                float* nb = B->box + 12 * (size_t)idx;
                for (int t = 0; t < 6; ++t) { nb[t] = a[t]; nb[6 + t] = b[t]; }
                B->child[2 * idx] = ref[i];
                B->child[2 * idx + 1] = ref[j];
                for (int t = 0; t < 3; ++t) { o[t] = fminf(a[t], b[t]); o[3 + t] = fmaxf(a[3 + t], b[3 + t]); }
                ref2[k++] = idx;
            } else {
                for (int t = 0; t < 6; ++t) o[t] = a[t];
                ref2[k++] = ref[i];
            }
        }
        next -= q;
        cnt = k;
        int* tr = ref; ref = ref2; ref2 = tr;
        float* tb = box; box = box2; box2 = tb;
    }
    free(ref); free(ref2); free(box); free(box2); free(nn);
}

/* Quantisation of the BVH4 child boxes (csrc/rr_device.h q4_exponent /
 * q4_quant, bvh.hip k_collapse4): per axis the smallest e in [-64, 100] with
 * 255 * 2^e >= the extent of the children's union (in double, exact), grid
 * origin = the union's lo corner, lo rounded down and hi up to [0, 255]. */
#define ORC_QEXP_MIN (-64)
#define ORC_QEXP_MAX 100
static int q4_exponent(double ext) {
    if (!(ext > 0.0)) return ORC_QEXP_MIN;
    int k;
    (void)frexp(ext, &k);
    int e = ldexp(255.0, k - 8) >= ext ? k - 8 : k - 7;
    return e < ORC_QEXP_MIN ? ORC_QEXP_MIN : (e > ORC_QEXP_MAX ? ORC_QEXP_MAX : e);
}
static uint32_t q4_quant(float v, float org, int e, int up) {
    double x = ((double)v - (double)org) * ldexp(1.0, -e);
    double q = up ? ceil(x) : floor(x);
    return q <= 0.0 ? 0u : (q >= 255.0 ? 255u : (uint32_t)q);
}
/* finite reciprocal for the quantised slab test (rr_device.h q4_rcp) */
static float q4_rcp(float x) { return fabsf(x) < 0x1p-64f ? (x < 0.0f ? -0x1p64f : 0x1p64f) : 1.0f / x; }
/* slab-test reciprocal of a direction (rr_device.h rcp3): one division when
 * the component product is at least 2^-100, else q4_rcp per component */
static v3 rcp3(v3 d) {
    float p = d.x * d.y;
    float q = p * d.z;
    if (fabsf(q) >= 0x1p-100f) {
        float r = 1.0f / q;
        return V(r * (d.y * d.z), r * (d.x * d.z), r * p);
    }
    return V(q4_rcp(d.x), q4_rcp(d.y), q4_rcp(d.z));
}

/* Quantised wide node (csrc/rr_device.h QNode6), 16 words = 64 B, up to six
 * children:
 *   w0..2  grid origin (float bits)   w3  exponent bytes (e + 128) per axis | inner mask << 24
 *   w4     index of the first internal child (the others follow in slot order)
 *   w5     position of the first leaf child's triangle (the others follow)
 *   w6..11 children 0..3: lo x, lo y, lo z, hi x, hi y, hi z (byte c = child c)
 *   w12..14 children 4, 5: (lo x, lo y), (lo z, hi x), (hi y, hi z) as byte pairs
 *   w15    mask of the used slots | the largest exponent byte << 8
 * An unused slot has lo 255, hi 0 on every axis and its bit of w15 clear: its
 * box test always fails. */
#define ORC_QW_MAX 6
#ifndef ORC_QW
#define ORC_QW 6 /* children per node (<= ORC_QW_MAX; rr_device.h kQWidth) */
#endif
/* sets grid coordinate `which` (0..2 lo x/y/z, 3..5 hi x/y/z) of child c */
static void qn_set_byte(uint32_t* w, int which, int c, uint32_t v) {
    if (c < 4) w[6 + which] |= v << (8 * c);
    else w[12 + which / 2] |= v << (16 * (which & 1) + 8 * (c - 4));
}
static void q4_pack(const float lo[3][ORC_QW_MAX], const float hi[3][ORC_QW_MAX], int used, uint32_t inner,
                    uint32_t inner_base, uint32_t tri_base, uint32_t* o) {
    uint32_t eb = 0;
    float org[3];
    memset(o, 0, 16 * sizeof(uint32_t));
    for (int a = 0; a < 3; ++a) {
        float l = lo[a][0], h = hi[a][0];
        for (int c = 1; c < used; ++c) { l = fminf(l, lo[a][c]); h = fmaxf(h, hi[a][c]); }
        int e = q4_exponent((double)h - (double)l);
        org[a] = l;
        eb |= (uint32_t)(e + 128) << (8 * a);
        for (int c = 0; c < ORC_QW_MAX; ++c) {
            qn_set_byte(o, a, c, c < used ? q4_quant(lo[a][c], l, e, 0) : 255u);
            qn_set_byte(o, 3 + a, c, c < used ? q4_quant(hi[a][c], l, e, 1) : 0u);
        }
    }
    memcpy(o, org, 3 * sizeof(float));
    o[3] = eb | inner << 24;
    o[4] = inner_base;
    o[5] = tri_base;
    {   /* used slots | the largest exponent byte << 8 (rr_device.h q6_planes' margin) */
        uint32_t emax = eb & 255u;
        if (((eb >> 8) & 255u) > emax) emax = (eb >> 8) & 255u;
        if (((eb >> 16) & 255u) > emax) emax = (eb >> 16) & 255u;
        o[15] = ((1u << used) - 1u) | emax << 8;
    }
}

/* BVH4 collapse of the BVH2 (PLOC, or Karras below 3 triangles), as
 * csrc/bvh.hip build_bvh4 (k_c4_count / k_c4_emit): breadth first from the
 * root; a node's children start as its BVH2 root's two children. A child
 * single triangle is a leaf entry (never opened);
 * while there are fewer than four entries, the internal entry with the
 * largest box measure dx*dy + dy*dz + dz*dx (ties: lowest slot) is replaced
 * by its left child and its right child appended. The internal children of a
 * node get consecutive indices in slot order after every node of the current
 * level (a FIFO numbering); the triangles of its leaf entries get consecutive
 * positions of the BVH4's own triangle array, in slot order and, within an
 * entry, in the left-first order of its subtree, after every triangle of the
 * levels before and of the nodes before it in its level (tri, tri_orig,
 * tri_mat are permuted into that order, so a leaf ref names the range
 * ~(first | (count - 1) << 28) of it). Boxes are the BVH2 child boxes,
 * quantised by q4_pack. */
typedef struct { int m; int ref[ORC_QW_MAX]; float lo[3][ORC_QW_MAX], hi[3][ORC_QW_MAX]; } c4set;

static void c4_put(const lbvh* B, c4set* S, int slot, int node, int side) {
    const float* f = B->box + 12 * (size_t)node + 6 * side;
    for (int a = 0; a < 3; ++a) { S->lo[a][slot] = f[a]; S->hi[a][slot] = f[3 + a]; }
    S->ref[slot] = B->n > 1 ? B->child[2 * node + side] : ~0;
}

/* an entry that stays a leaf: one triangle (the product's leaves hold one) */
static int c4_leaf(const c4set* S, int c) { return S->ref[c] < 0; }

static void c4_set(const lbvh* B, int r, c4set* S) {
    c4_put(B, S, 0, r, 0);
    c4_put(B, S, 1, r, 1);
    S->m = B->n > 1 ? 2 : 1; /* one triangle: one leaf slot */
    while (S->m < ORC_QW) {
        int best = -1;
        float ba = 0.0f;
        for (int c = 0; c < S->m; ++c) {
            if (c4_leaf(S, c)) continue;
            float dx = S->hi[0][c] - S->lo[0][c], dy = S->hi[1][c] - S->lo[1][c], dz = S->hi[2][c] - S->lo[2][c];
            float a = dx * dy + dy * dz + dz * dx;
            if (best < 0 || a > ba) { best = c; ba = a; }
        }
        if (best < 0) break;
        int cn = S->ref[best];
        c4_put(B, S, S->m, cn, 1);
        c4_put(B, S, best, cn, 0);
        ++S->m;
    }
}

/* Research switch (tools/collapse_study.py, not the product): 1 = the wide
 * nodes chosen by a surface-area dynamic programme over the BVH2 (Ylitie et
 * al. 2017) instead of the greedy opening of c4_set. */
static int g_collapse;
void orc_set_collapse(int mode) { g_collapse = mode; }
static double box_area_d(const float* b) {
    double dx = (double)b[3] - b[0], dy = (double)b[4] - b[1], dz = (double)b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
}
/* dp_dist[6 n + j - 1] = least cost of covering BVH2 subtree n with at most j
 * entries of a wide node; dp_pick[6 n + j - 1] = 0: n itself is the entry,
 * a > 0: a entries for the left child, j - a for the right; dp_root[n] = the
 * left child's share when n is a wide node. */
static double* dp_dist;
static unsigned char *dp_pick, *dp_root;
static double dp_child(const lbvh* B, int ref, int j) { return ref < 0 ? 0.0 : dp_dist[6 * (size_t)ref + j - 1]; }
static void dp_build(const lbvh* B) {
    const int ni = B->n - 1;
    dp_dist = (double*)malloc(sizeof(double) * 6 * (size_t)ni);
    dp_pick = (unsigned char*)malloc(6 * (size_t)ni);
    dp_root = (unsigned char*)malloc((size_t)ni);
    for (int v = ni - 1; v >= 0; --v) {  /* PLOC: children have larger indices */
        const int l = B->child[2 * v], r = B->child[2 * v + 1];
        float box[6];
        for (int a = 0; a < 3; ++a) {
            box[a] = fminf(B->box[12 * (size_t)v + a], B->box[12 * (size_t)v + 6 + a]);
            box[3 + a] = fmaxf(B->box[12 * (size_t)v + 3 + a], B->box[12 * (size_t)v + 9 + a]);
        }
        double best = INFINITY;
        int ba = 1;
        for (int a = 1; a <= 5; ++a) {
            double c = dp_child(B, l, a) + dp_child(B, r, 6 - a);
            if (c < best) { best = c; ba = a; }
        }
        const double own = box_area_d(box) + best;
        dp_root[v] = (unsigned char)ba;
        for (int j = 1; j <= 6; ++j) {
            double bj = own;
            int pick = 0;
            for (int a = 1; a < j; ++a) {
                double c = dp_child(B, l, a) + dp_child(B, r, j - a);
                if (c < bj) { bj = c; pick = a; }
            }
            dp_dist[6 * (size_t)v + j - 1] = bj;
            dp_pick[6 * (size_t)v + j - 1] = (unsigned char)pick;
        }
    }
}
static void dp_expand(const lbvh* B, int v, int side, int j, c4set* S) {
    const int ref = B->child[2 * v + side];
    if (ref >= 0 && dp_pick[6 * (size_t)ref + j - 1] != 0) {
        const int a = dp_pick[6 * (size_t)ref + j - 1];
        dp_expand(B, ref, 0, a, S);
        dp_expand(B, ref, 1, j - a, S);
        return;
    }
    c4_put(B, S, S->m++, v, side);
}

static void lbvh_collapse4(lbvh* B) {
    const int n = B->n;
    B->n4 = 0;
    if (n <= 0) return;
    const int dp = g_collapse == 1 && n > 2;
    if (dp) dp_build(B);
    const int ni = n > 1 ? n - 1 : 1;
    int* src = (int*)malloc(sizeof(int) * (size_t)ni);
    int* perm = (int*)malloc(sizeof(int) * (size_t)n);  /* BVH4 triangle position -> sorted leaf */
    B->child4 = (int*)malloc(sizeof(int) * ORC_QW_MAX * (size_t)ni);
    B->q4 = (uint32_t*)malloc(sizeof(uint32_t) * 16 * (size_t)ni);
    src[0] = 0;
    int count = 1, ntri = 0;
    for (int idx = 0; idx < count; ++idx) {
        c4set S;
        if (dp) {
            const int a = dp_root[src[idx]];
            S.m = 0;
            dp_expand(B, src[idx], 0, a, &S);
            dp_expand(B, src[idx], 1, 6 - a, &S);
        } else {
            c4_set(B, src[idx], &S);
        }
        int ref[ORC_QW_MAX];
        uint32_t inner = 0;
        const int inner_base = count, tri_base = ntri;
        for (int c = 0; c < ORC_QW_MAX; ++c) {
            if (c >= S.m) ref[c] = ORC_EMPTY4;
            else if (!c4_leaf(&S, c)) { src[count] = S.ref[c]; ref[c] = count++; inner |= 1u << c; }
            else if (n == 1) { perm[0] = 0; ref[c] = leaf_ref(0, 1); ntri = 1; }
            else { /* a leaf entry is one triangle: position ntri */
                perm[ntri] = ~S.ref[c];
                ref[c] = leaf_ref(ntri, 1);
                ntri += 1;
            }
        }
        q4_pack((const float(*)[ORC_QW_MAX])S.lo, (const float(*)[ORC_QW_MAX])S.hi, S.m, inner, (uint32_t)inner_base,
                (uint32_t)tri_base, B->q4 + 16 * (size_t)idx);
        for (int c = 0; c < ORC_QW_MAX; ++c) B->child4[ORC_QW_MAX * (size_t)idx + c] = ref[c];
    }
    B->n4 = count;
    /* the triangle arrays in the BVH4's leaf order */
    float* tri = (float*)malloc(sizeof(float) * 9 * (size_t)n);
    int* orig = (int*)malloc(sizeof(int) * (size_t)n);
    int* mat = (int*)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        memcpy(tri + 9 * (size_t)i, B->tri + 9 * (size_t)perm[i], 9 * sizeof(float));
        orig[i] = B->tri_orig[perm[i]];
        mat[i] = B->tri_mat[perm[i]];
    }
    free(B->tri); free(B->tri_orig); free(B->tri_mat);
    B->tri = tri; B->tri_orig = orig; B->tri_mat = mat;
    free(src); free(perm);
    if (dp) { free(dp_dist); free(dp_pick); free(dp_root); }
}

/* ------------------------------------------------------------ tracing ---- */
typedef struct { float t, u, v; int idx, orig; } hitrec;

/* Watertight traversal (csrc/rr_device.h, "intersection"): the triangle test
 * decides a hit exactly in a 2D projection of the ray's own (woop_test), and
 * every box test widens the box by ORC_BOX_MARGIN (2^-19) of the largest
 * coordinate involved — a distance along each axis, margin * |1/d| in t:
 * subtracted from the near planes, added to the far ones. The BVH2 walk takes
 * it per ray (|o|_inf + the scene box's largest |coordinate|), the quantised
 * walk per node (the node's largest |org - o| + extent, q6_planes). */
#define ORC_BOX_MARGIN 0x1p-19f

/* plane distances fmaf(b, inv, oi), oi = -(o inv) per ray, widened by em per
 * axis (rr_device.h slab) */
static int slab_test(v3 oi, v3 inv, v3 em, const float* b, float tmin, float tmax, float* tnear) {
    float tx0 = fmaf(b[0], inv.x, oi.x), tx1 = fmaf(b[3], inv.x, oi.x);
    float ty0 = fmaf(b[1], inv.y, oi.y), ty1 = fmaf(b[4], inv.y, oi.y);
    float tz0 = fmaf(b[2], inv.z, oi.z), tz1 = fmaf(b[5], inv.z, oi.z);
    float tn = fmaxf(fmaxf(fminf(tx0, tx1) - em.x, fminf(ty0, ty1) - em.y), fmaxf(fminf(tz0, tz1) - em.z, tmin));
    float tf = fminf(fminf(fmaxf(tx0, tx1) + em.x, fmaxf(ty0, ty1) + em.y), fminf(fmaxf(tz0, tz1) + em.z, tmax));
    *tnear = tn;
    return tn <= tf;
}
/* BVH2 margins of one ray (rr_device.h slab_margin): ORC_BOX_MARGIN (|o|_inf +
 * r) |1/d| per axis, r = the largest |coordinate| of the scene box */
static v3 slab_margin(v3 o, v3 inv, float r) {
    float m = (fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) + r) * ORC_BOX_MARGIN;
    return V(m * fabsf(inv.x), m * fabsf(inv.y), m * fabsf(inv.z));
}
/* rr_device.h scene_radius: over the root's 12 box floats, the same fmaxf tree */
static float scene_radius(const float* r) {
    float a = fmaxf(fmaxf(fmaxf(fabsf(r[0]), fabsf(r[1])), fmaxf(fabsf(r[2]), fabsf(r[3]))), fmaxf(fabsf(r[4]), fabsf(r[5])));
    float b = fmaxf(fmaxf(fmaxf(fabsf(r[6]), fabsf(r[7])), fmaxf(fabsf(r[8]), fabsf(r[9]))), fmaxf(fabsf(r[10]), fabsf(r[11])));
    return fmaxf(a, b);
}

/* Watertight ray/triangle test (Woop, Benthin & Wald, JCGT 2(1) 2013), as
 * rr_device.h make_shear / woop_core: per ray kz = the axis of the largest |d|
 * component (ties: x before y before z), (kx, ky) = (kz + 1, kz + 2) mod 3,
 * sz = 1 / d[kz], sx = d[kx] sz, sy = d[ky] sz; per triangle the vertices
 * relative to the origin, permuted, sheared to x = a[kx] - sx a[kz],
 * y = a[ky] - sy a[kz]; edge functions U = cx by - cy bx, V = ax cy - ay cx,
 * W = bx ay - by ax (no contraction: a shared edge gives exactly opposite
 * values; one that rounds to 0 recomputed exactly, edge_exact); hit iff no two
 * of them have opposite signs and det = U + V + W != 0; t = (U sz az + V sz bz
 * + W sz cz) / det, u = V / det, v = W / det. */
typedef struct { float sx, sy, sz; int kz; } shear_t;
static v3 rot3(v3 a, int kz) {
    int k0 = kz == 0, k1 = kz == 1;
    return V(k0 ? a.y : (k1 ? a.z : a.x), k0 ? a.z : (k1 ? a.x : a.y), k0 ? a.x : (k1 ? a.y : a.z));
}
static shear_t make_shear(v3 d) {
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    shear_t s;
    s.kz = ax >= ay ? (ax >= az ? 0 : 2) : (ay >= az ? 1 : 2);
    v3 r = rot3(d, s.kz);
    s.sz = 1.0f / r.z;
    s.sx = r.x * s.sz;
    s.sy = r.y * s.sz;
    return s;
}
static float edge_exact(float a, float b, float c, float d, float e) {
    if (e != 0.0f) return e;
    return fmaf(a, b, -(a * b)) - fmaf(c, d, -(c * d));
}
static int woop_test(const shear_t* s, v3 o, const float* t9, float* t, float* u, float* v) {
    v3 a = rot3(vsub(V(t9[0], t9[1], t9[2]), o), s->kz);
    v3 b = rot3(vsub(V(t9[3], t9[4], t9[5]), o), s->kz);
    v3 c = rot3(vsub(V(t9[6], t9[7], t9[8]), o), s->kz);
    float ax = fmaf(-s->sx, a.z, a.x), ay = fmaf(-s->sy, a.z, a.y);
    float bx = fmaf(-s->sx, b.z, b.x), by = fmaf(-s->sy, b.z, b.y);
    float cx = fmaf(-s->sx, c.z, c.x), cy = fmaf(-s->sy, c.z, c.y);
    float U = cx * by - cy * bx;
    float Vv = ax * cy - ay * cx;
    float W = bx * ay - by * ax;
    if (U == 0.0f || Vv == 0.0f || W == 0.0f) {
        U = edge_exact(cx, by, cy, bx, U);
        Vv = edge_exact(ax, cy, ay, cx, Vv);
        W = edge_exact(bx, ay, by, ax, W);
    }
    float det = U + Vv + W;
    float mn = fminf(fminf(U, Vv), W), mx = fmaxf(fmaxf(U, Vv), W);
    if ((mn < 0.0f && mx > 0.0f) || det == 0.0f) return 0;
    float T = fmaf(W, s->sz * c.z, fmaf(Vv, s->sz * b.z, U * (s->sz * a.z)));
    float inv = 1.0f / det;
    *t = T * inv;
    *u = Vv * inv;
    *v = W * inv;
    return 1;
}

static void try_leaf(const lbvh* B, int leaf, const shear_t* s, v3 o, float tmin, hitrec* h) {
    float t, u, v;
    if (!woop_test(s, o, B->tri + 9 * (size_t)leaf, &t, &u, &v)) return;
    int orig = B->tri_orig[leaf];
    if (t > tmin && (t < h->t || (t == h->t && orig < h->orig))) {
        h->t = t; h->u = u; h->v = v; h->idx = leaf; h->orig = orig;
    }
}

typedef struct { float t; int slot, ref; } ckey;

#ifdef ORC_WALK_STUDY
/* research build only: [0] node visits whose entry distance (as tested at the
 * parent) exceeds the closest hit at visit time, [1] grouped-entry pops whose
 * every child lies beyond it */
static long long g_cnt_study[2];
static int g_study_order; /* 1: grouped entries pop nearest first; 2: and skip children beyond the hit */
void orc_study_order(int mode) { g_study_order = mode; }
void orc_walk_study(long long* out2, int reset) {
    out2[0] = g_cnt_study[0]; out2[1] = g_cnt_study[1];
    if (reset) g_cnt_study[0] = g_cnt_study[1] = 0;
}
#endif

/* node visits / triangle tests of trace4 since the last reset (research:
 * tools/collapse_study.py, tools/margin_study.py). Counted only while a study
 * tool has switched counting on (orc_set_walk_counting): the shared totals are
 * updated atomically once per ray, which would otherwise put every render
 * thread on one cache line (and slow the CPU baseline). */
static long long g_cnt_nodes, g_cnt_tris, g_cnt_top[4];
static int g_count_walks;
void orc_set_walk_counting(int on) { g_count_walks = on; }
/* research only (tools/margin_study.py): the walk's box margin times this
 * (1 = the product's); results then may differ from the device's */
static float g_margin_scale = 1.0f;
void orc_set_margin_scale(float s) { g_margin_scale = s; }
/* out: node visits, triangle tests, visits of nodes below 128 / 256 / 512 / 1024 */
void orc_walk_counts(long long* out6, int reset) {
    out6[0] = g_cnt_nodes; out6[1] = g_cnt_tris;
    for (int k = 0; k < 4; ++k) out6[2 + k] = g_cnt_top[k];
    if (reset) { g_cnt_nodes = g_cnt_tris = 0; for (int k = 0; k < 4; ++k) g_cnt_top[k] = 0; }
}

/* traversal-stack pushes dropped for want of room (ORC_MAXDEPTH), since the
 * last orc_reset_stack_drops: each a missed subtree, as on the GPU
 * (rr_frame_stats.stack_drops) */
static long long g_drops;
static void drop_push(void) {
#pragma omp atomic
    g_drops += 1;
}
long long orc_stack_drops(void) { return g_drops; }
void orc_reset_stack_drops(void) { g_drops = 0; }

/* Quantised wide walk of rr_device.h TravStateQW: per axis s = iq * 2^e,
 * o' = (org - o) * iq, plane t = fma(q, s, o'), near plane lo for iq >= 0 else
 * hi; the ORC_QW_MAX box tests against the bound at node entry (unused slots
 * always fail), passing leaf children intersected in slot order, the nearest
 * hit internal child (ties: lower slot) visited next, the other hit internal
 * children pushed in descending slot order. Child refs are implicit: internal
 * child c is node w4 + (internal slots before c), leaf child c is triangle
 * w5 + (leaf slots before c). */
static int trace4(const lbvh* B, v3 o, v3 d, float tmin, float tmax, int any, hitrec* h) {
    h->t = tmax; h->u = h->v = 0.0f; h->idx = -1; h->orig = -1;
    if (B->n <= 0) return 0;
    const shear_t sh = make_shear(d);
    const v3 iqv = rcp3(d);
    const float iq[3] = {iqv.x, iqv.y, iqv.z};
    const float oo[3] = {o.x, o.y, o.z};
    int stack[ORC_MAXDEPTH];
    int sp = 0, node = 0;
    long long cn = 0, ct = 0, ctop[4] = {0, 0, 0, 0};
#ifdef ORC_WALK_STUDY
    /* research build only (tools/walk_study.py): the entry distance of every
     * stacked child, to count the visits a pop-time test against the current
     * closest hit would skip */
    float stk_t[ORC_MAXDEPTH][ORC_QW_MAX];
    float node_t = -INFINITY;
    long long cull = 0, cull_grp = 0;
#endif
    for (;;) {
#ifdef ORC_WALK_STUDY
        if (node_t > h->t) ++cull;
#endif
        ++cn;
        for (int k = 0; k < 4; ++k) ctop[k] += node < (128 << k);
        const uint32_t* nd = B->q4 + 16 * (size_t)node;
        const uint32_t inner = nd[3] >> 24;
        const float tcur = h->t;
        float sc[3], onr[3], ofr[3];
        int pos[3];
        /* rr_device.h q6_planes: the node's margin distance ORC_BOX_MARGIN (the
         * largest |org - o| + 255 * 2^(the largest e)) */
        float dif[3];
        for (int a = 0; a < 3; ++a) {
            float org;
            memcpy(&org, nd + a, sizeof org);
            const int e = (int)((nd[3] >> (8 * a)) & 255u) - 128;
            dif[a] = org - oo[a];
            sc[a] = ldexpf(iq[a], e);
        }
        const float M = ORC_BOX_MARGIN * g_margin_scale;
        const float mrg = fmaf(fmaxf(fmaxf(fabsf(dif[0]), fabsf(dif[1])), fabsf(dif[2])), M,
                               ldexpf(255.0f * M, (int)((nd[15] >> 8) & 255u) - 128));
        for (int a = 0; a < 3; ++a) {
            const float ma = mrg * fabsf(iq[a]);
            onr[a] = fmaf(dif[a], iq[a], -ma);
            ofr[a] = fmaf(dif[a], iq[a], ma);
            pos[a] = iq[a] >= 0.0f;
        }
        /* near / far grid coordinates per axis: children 0..3 one byte of a
         * word, 4 and 5 a byte pair */
        uint32_t nw[3], fw[3], nw2[3], fw2[3];
        for (int a = 0; a < 3; ++a) {
            const uint32_t lo = nd[6 + a], hi = nd[9 + a];
            const uint32_t lo2 = (nd[12 + a / 2] >> (16 * (a & 1))) & 0xffffu;
            const uint32_t hi2 = (nd[12 + (3 + a) / 2] >> (16 * ((3 + a) & 1))) & 0xffffu;
            nw[a] = pos[a] ? lo : hi; fw[a] = pos[a] ? hi : lo;
            nw2[a] = pos[a] ? lo2 : hi2; fw2[a] = pos[a] ? hi2 : lo2;
        }
        ckey k[ORC_QW_MAX];
        int n_in = 0, n_lf = 0;
        for (int c = 0; c < ORC_QW_MAX; ++c) {
            float p0[3], p1[3];
            for (int a = 0; a < 3; ++a) {
                const uint32_t qn = c < 4 ? (nw[a] >> (8 * c)) & 255u : (nw2[a] >> (8 * (c - 4))) & 255u;
                const uint32_t qf = c < 4 ? (fw[a] >> (8 * c)) & 255u : (fw2[a] >> (8 * (c - 4))) & 255u;
                p0[a] = fmaf((float)qn, sc[a], onr[a]);
                p1[a] = fmaf((float)qf, sc[a], ofr[a]);
            }
            const float tn = fmaxf(fmaxf(p0[0], p0[1]), fmaxf(p0[2], tmin));
            const float tf = fminf(fminf(p1[0], p1[1]), fminf(p1[2], tcur));
            const int is_inner = (inner >> c) & 1u;
            const int ref = is_inner ? (int)nd[4] + n_in : ~((int)nd[5] + n_lf);
            if (is_inner) ++n_in; else ++n_lf;
            const int hit = tn <= tf && ((nd[15] >> c) & 1u);
            k[c].slot = c;
            k[c].ref = ref;
            k[c].t = (hit && is_inner) ? tn : INFINITY;
            if (hit && !is_inner) {
                ++ct;
                try_leaf(B, ~ref, &sh, o, tmin, h);
                if (any && h->idx >= 0) goto done;
            }
        }
        /* nearest hit internal child next (ties: lower slot; any-hit rays:
         * the lowest hit internal slot); the others are pushed in descending
         * slot order */
        int best = -1;
        for (int c = 0; c < ORC_QW_MAX; ++c)
            if (k[c].t != INFINITY && (best < 0 || (!any && k[c].t < k[best].t))) best = c;
        if (best < 0) {
#ifdef ORC_WALK_STUDY
        pop_again:
#endif
            if (sp == 0) break;
            /* grouped entries (rr_device.h TravStackT::pop_group): the lowest
             * rank left; the entry stays while ranks remain */
            const int e = stack[sp - 1];
            int r = 0;
            while (!((e >> r) & 1)) ++r;
#ifdef ORC_WALK_STUDY
            if (g_study_order)  /* research: the entry's nearest child first */
                for (int q = r + 1; q < ORC_QW_MAX; ++q)
                    if (((e >> q) & 1) && stk_t[sp - 1][q] < stk_t[sp - 1][r]) r = q;
#endif
            node = (int)((unsigned)e >> 6) + r;
#ifdef ORC_WALK_STUDY
            node_t = stk_t[sp - 1][r];
            if (g_study_order > 1 && node_t > h->t) {  /* research: skip what lies beyond the hit */
                const int rest2 = e & ~(1 << r);
                if ((rest2 & 63) == 0) --sp; else stack[sp - 1] = rest2;
                goto pop_again;
            }
            {
                float mn = INFINITY;
                for (int q = 0; q < ORC_QW_MAX; ++q)
                    if ((e >> q) & 1) mn = fminf(mn, stk_t[sp - 1][q]);
                if (mn > h->t) ++cull_grp;  /* the whole entry beyond the hit: one pop for all its children */
            }
#endif
#ifdef ORC_WALK_STUDY
            const int rest = e & ~(1 << r);
#else
            const int rest = e & (e - 1);
#endif
            if ((rest & 63) == 0) --sp; else stack[sp - 1] = rest;
            continue;
        }
        /* the other hit internal children as one entry: the node's first
         * internal child << 6 | their ranks among its internal children (they
         * come off in slot order, as single pushes in descending slot order
         * would give; node indices below 2^26, as the device build checks) */
        {
            unsigned rm = 0;
            for (int c = 0, rank = 0; c < ORC_QW_MAX; ++c) {
                if (!((inner >> c) & 1u)) continue;
                if (c != best && k[c].t != INFINITY) rm |= 1u << rank;
                ++rank;
            }
            if (rm) {
#ifdef ORC_WALK_STUDY
                if (sp < ORC_MAXDEPTH)
                    for (int c = 0, rank = 0; c < ORC_QW_MAX; ++c) {
                        if (!((inner >> c) & 1u)) continue;
                        stk_t[sp][rank++] = k[c].t;
                    }
#endif
                if (sp < ORC_MAXDEPTH) stack[sp++] = (int)((nd[4] << 6) | rm);
                else drop_push();
            }
        }
        node = k[best].ref;
#ifdef ORC_WALK_STUDY
        node_t = k[best].t;
#endif
    }
done:
#ifdef ORC_WALK_STUDY
    if (g_count_walks) {
#pragma omp atomic
        g_cnt_study[0] += cull;
#pragma omp atomic
        g_cnt_study[1] += cull_grp;
    }
#endif
    if (g_count_walks) {
        for (int k = 0; k < 4; ++k) {
#pragma omp atomic
            g_cnt_top[k] += ctop[k];
        }
#pragma omp atomic
        g_cnt_nodes += cn;
#pragma omp atomic
        g_cnt_tris += ct;
    }
    return h->idx >= 0;
}

/* Same traversal order as the GPU (near child first, left on ties, leaves
 * tested as soon as their box passes). */
static int trace(const lbvh* B, v3 o, v3 d, float tmin, float tmax, int any, hitrec* h) {
    if (B->width == 4) return trace4(B, o, d, tmin, tmax, any, h);
    h->t = tmax; h->u = h->v = 0.0f; h->idx = -1; h->orig = -1;
    if (B->n <= 0) return 0;
    const shear_t sh = make_shear(d);
    v3 inv = rcp3(d);
    v3 oi = V(-(o.x * inv.x), -(o.y * inv.y), -(o.z * inv.z));
    v3 em = slab_margin(o, inv, scene_radius(B->box));
    int stack[ORC_MAXDEPTH];
    int sp = 0, node = 0;
    for (;;) {
        const float* bx = B->box + 12 * (size_t)node;
        float tl, tr;
        int hl = slab_test(oi, inv, em, bx, tmin, h->t, &tl);
        int hr = slab_test(oi, inv, em, bx + 6, tmin, h->t, &tr);
        int cl = B->child_lf[2 * node], cr = B->child_lf[2 * node + 1];
        int nl = 0, nr = 0, fl = 0, fr = 0;
        if (hl && cl < 0) { fl = leaf_first(cl); nl = leaf_count(cl); hl = 0; }
        if (hr && cr < 0) { fr = leaf_first(cr); nr = leaf_count(cr); hr = 0; }
        for (int k = 0; k < nl + nr; ++k) {
            try_leaf(B, k < nl ? fl + k : fr + (k - nl), &sh, o, tmin, h);
            if (any && h->idx >= 0) return 1;
        }
        if (hl && hr) {
            int lf = tl <= tr;
            if (sp < ORC_MAXDEPTH) stack[sp++] = lf ? cr : cl;
            else drop_push();
            node = lf ? cl : cr;
        } else if (hl) node = cl;
        else if (hr) node = cr;
        else {
            if (sp == 0) break;
            node = stack[--sp];
        }
    }
    return h->idx >= 0;
}

/* ------------------------------------------------------------ material ---- */
/* Blender 3.6 Cycles' Principled BSDF v1 for the subset the scenes use (base,
 * metallic, specular, roughness), restated from Cycles (third-party, not in
 * /root/reference): closure setup in intern/cycles/kernel/svm/closure.h
 * (CLOSURE_BSDF_PRINCIPLED_ID: cspec0, ior = 2/(1 - sqrt(0.08 specular)) - 1,
 * closures present above CLOSURE_WEIGHT_CUTOFF 1e-5), the diffuse closure of
 * bsdf_principled_diffuse.h (PRINCIPLED_DIFFUSE_FULL), and the GGX closure
 * with Fresnel of bsdf_microfacet.h (interpolate_fresnel_color,
 * fresnel_dielectric_cos of bsdf_util.h; sample weight scaled by the average
 * Fresnel colour at the view angle). Same float operations as
 * csrc/rr_device.h mat_derive / bsdf_eval_v / bsdf_view / bsdf_sample; the
 * Fresnel blend and the lobe pick probability are read from per-material
 * tables built in double exactly as csrc/scene.cpp build_material_lut. */
typedef struct { v3 base; float metallic, specular, roughness, ior; v3 emission; int model; } mat_t;

#define ORC_LUT_N 128
#define ORC_LUT_STRIDE 260

static float sw(float c) { float m = 1.0f - c; if (m < 0.0f) m = 0.0f; float m2 = m * m; return m2 * m2 * m; }

static double fresnel_dielectric_d(double cosi, double eta) {
    double c = fabs(cosi);
    double g = eta * eta - 1.0 + c * c;
    if (g > 0.0) {
        g = sqrt(g);
        double A = (g - c) / (g + c);
        double B = (c * (g + c) - 1.0) / (c * (g - c) + 1.0);
        return 0.5 * A * A * (1.0 + B * B);
    }
    return 1.0;
}

static double clamp01d(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }

/* FH(cos of the half angle) [0, 128] + [128] repeated | spec pick probability(cos of
 * the view) [130, 258] + [258] repeated (csrc/scene.cpp build_material_lut) */
#define ORC_LUT_PS 130
void orc_material_lut(const float* m, float* out) {
    const int N = ORC_LUT_N;
    double spec = m[4], met = m[3];
    double b[3] = {m[0], m[1], m[2]};
    int model = (int)m[10];
    int spec_on = m[4] > 1.0e-5f || m[3] > 1.0e-5f;
    double eta = 2.0 / (1.0 - sqrt(0.08 * spec)) - 1.0;
    double f0 = fresnel_dielectric_d(1.0, eta);
    double c0[3];
    for (int k = 0; k < 3; ++k) c0[k] = clamp01d(spec * 0.08 * (1.0 - met) + b[k] * met);
    double wd = (1.0 - met) * ((b[0] + b[1] + b[2]) / 3.0);
    for (int i = 0; i <= N; ++i) {
        double c = (double)i / N;
        out[i] = (float)((fresnel_dielectric_d(c, eta) - f0) / (1.0 - f0));
    }
    for (int i = 0; i <= N; ++i) {
        double c = (double)i / N;
        double fh = (fresnel_dielectric_d(c, eta) - f0) / (1.0 - f0);
        double wsp = ((c0[0] * (1.0 - fh) + fh) + (c0[1] * (1.0 - fh) + fh) + (c0[2] * (1.0 - fh) + fh)) / 3.0;
        double ps = 0.0;
        if (model != 1 && spec_on) ps = wsp + wd > 0.0 ? wsp / (wsp + wd) : 1.0;
        out[ORC_LUT_PS + i] = (float)ps;
    }
    out[N + 1] = out[N];
    out[ORC_LUT_PS + N + 1] = out[ORC_LUT_PS + N];
}

static float lut_at(const float* t, float u) {
    u = fminf(fmaxf(u, 0.0f), 1.0f);
    return lerp_table(t, ORC_LUT_N + 1, u);
}

static float sat1(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

/* terms Cycles derives at closure setup */
typedef struct { float alpha, a2, kd0; v3 cspec0; int spec_on; } mterms;

static mterms mat_terms(const mat_t* m) {
    mterms t;
    float alpha = m->roughness * m->roughness;
    if (alpha < 1.0e-3f) alpha = 1.0e-3f;  /* see csrc/rr_device.h mat_derive */
    t.alpha = alpha;
    t.a2 = alpha * alpha;
    float sm = m->specular * 0.08f * (1.0f - m->metallic);
    t.cspec0 = V(sat1(sm + m->base.x * m->metallic), sat1(sm + m->base.y * m->metallic),
                 sat1(sm + m->base.z * m->metallic));
    t.kd0 = (1.0f - m->metallic) * 0.318309886183791f;
    t.spec_on = (m->specular > 1.0e-5f || m->metallic > 1.0e-5f) ? 1 : 0;
    return t;
}

/* c + sqrt(a2 + (1 - a2) c^2): Smith G1(c) = 2c / c1 */
static float g1_den(float a2, float c) { return c + sqrtf(fmaf((1.0f - a2) * c, c, a2)); }

/* f * cosL and the combined pdf (csrc/rr_device.h bsdf_eval_v, one division:
 * den = 2 + 2 L.V, X = (cosV + cosL)^2 (a2 - 1) + den = tt den,
 * pdf_s = a2 den^2 / (2 pi X^2 cv1), ks = a2 den^2 cosL / (pi X^2 cv1 cl1)) */
static v3 eval_bsdf(const mat_t* m, const float* lut, v3 N, v3 wo, v3 wi, float ps, float* pdf) {
    float cosV = vdot(N, wo), cosL = vdot(N, wi);
    if (cosV <= 0.0f || cosL <= 0.0f) { *pdf = 0.0f; return V(0.0f, 0.0f, 0.0f); }
    if (m->model == 1) { /* pure Lambert */
        *pdf = cosL * 0.318309886183791f;
        return vscl(m->base, *pdf);
    }
    mterms T = mat_terms(m);
    float lv = vdot(wi, wo);
    float a2 = T.a2;
    float fl = sw(cosL), fv = sw(cosV);
    float rr = m->roughness * (lv + 1.0f);
    float kd = T.kd0 * fmaf(rr, fmaf(fl * fv, rr - 1.0f, fl + fv), fmaf(-0.5f, fv, 1.0f) * fmaf(-0.5f, fl, 1.0f)) * cosL;
    float sv = cosV + cosL;
    float den = fmaf(2.0f, lv, 2.0f);
    float X = fmaf(sv * sv, a2 - 1.0f, den);
    float cv1 = g1_den(a2, cosV), cl1 = g1_den(a2, cosL);
    float q = a2 * den * den;
    float r = 1.0f / (3.14159265358979f * X * X * cv1 * cl1);
    float pdf_s = q * cl1 * r * 0.5f;
    float ks = T.spec_on ? q * cosL * r : 0.0f;
    float fh = lut_at(lut, sqrtf(fmaf(0.5f, lv, 0.5f)));
    v3 c0 = T.cspec0;
    float fh1 = 1.0f - fh;
    v3 F = V(fmaf(c0.x, fh1, fh), fmaf(c0.y, fh1, fh), fmaf(c0.z, fh1, fh));
    float pdf_d = cosL * 0.318309886183791f;
    *pdf = fmaf(ps, pdf_s, (1.0f - ps) * pdf_d);
    return V(fmaf(F.x, ks, m->base.x * kd), fmaf(F.y, ks, m->base.y * kd), fmaf(F.z, ks, m->base.z * kd));
}

static float p_spec(const float* lut, float cosV) { return lut_at(lut + ORC_LUT_PS, cosV); }

/* GGX visible normals by spherical caps (Dupuy & Benyoub 2023), csrc/rr_device.h sample_vndf */
static v3 vndf(v3 v, float alpha, float dx, float dy) {
    v3 vh = vnorm(V(alpha * v.x, alpha * v.y, v.z));
    float r2 = fmaf(dy, dy, dx * dx);
    float k = 1.0f + vh.z;
    float z = fmaf(-r2, k, 1.0f);
    float s = sqrtf(fmaxf(0.0f, k * fmaf(-r2, k, 2.0f)));
    v3 h = V(fmaf(dx, s, vh.x), fmaf(dy, s, vh.y), fmaxf(0.0f, z + vh.z));
    return vnorm(V(alpha * h.x, alpha * h.y, h.z));
}

/* glossy: the specular lobe was picked (Cycles LABEL_GLOSSY, else LABEL_DIFFUSE); f = f * cosL */
static int sample_bsdf(const mat_t* m, const float* lut, v3 N, v3 wo, float ul, float u1, float u2, v3* wi, v3* f,
                       float* pdf, int* glossy) {
    float cosV = vdot(N, wo);
    if (cosV <= 0.0f) return 0;
    float ps = p_spec(lut, cosV);
    v3 T, B;
    onb(N, &T, &B);
    float x, y;
    disk(u1, u2, &x, &y);
    *glossy = ul < ps;
    if (ul < ps) {
        float alpha = m->roughness * m->roughness;
        if (alpha < 1.0e-3f) alpha = 1.0e-3f;
        v3 wl = V(vdot(wo, T), vdot(wo, B), cosV);
        v3 hl = vndf(wl, alpha, x, y);
        v3 H = vframe(T, B, N, hl.x, hl.y, hl.z);
        float k = 2.0f * vdot(wo, H);
        *wi = V(fmaf(H.x, k, -wo.x), fmaf(H.y, k, -wo.y), fmaf(H.z, k, -wo.z));
    } else {
        float z = sqrtf(fmaxf(0.0f, fmaf(-y, y, fmaf(-x, x, 1.0f))));
        *wi = vframe(T, B, N, x, y, z);
    }
    *f = eval_bsdf(m, lut, N, wo, *wi, ps, pdf);
    return *pdf > 0.0f;
}

static v3 clampc(v3 c, float clamp) {
    if (clamp > 0.0f) {
        float mx = vmax3(c);
        if (mx > clamp) return vscl(c, clamp / mx);
    }
    return c;
}

/* ------------------------------------------------------------- render ---- */
typedef struct {
    const lbvh* bvh;
    const float* cam;     /* 16 */
    int n_lights;
    const float* lights;  /* 12 each */
    const float* mats;    /* 12 each */
    v3 world;
    int W, H, spp, max_bounces, view;
    int max_diffuse, max_glossy;  /* Cycles per-lobe bounce caps (>= 1) */
    float* luts;                  /* ORC_LUT_STRIDE floats per material */
    uint32_t seed;
    float clamp, inv_w2, inv_h2;
    float filter[ORC_FILTER_N];
    float srgb[ORC_SRGB_N + 1];
    int cam_all;          /* camera rays test every triangle (LDS-resident scenes, render_ints[7] == 2) */
    unsigned char* hull;  /* LDS-resident scenes: per leaf, bit 0 / 1 = the scene lies behind its front / back side (tri_hull) */
    int cull_on;          /* screen_rect() succeeded */
    float cull[4];        /* x0 x1 y0 y1 in subpixel coordinates */
} scene_t;

/* Screen-space bounds of the scene box, as rr_device.h screen_rect (same
 * float operations): the 8 corners projected to camera_ray's subpixel
 * coordinates, bounding rectangle widened by one pixel; 0 if a corner is not
 * at least 1e-4 in front of the camera. A camera ray outside it misses. */
static int screen_rect(const float* c, float W, float H, const float lo[3], const float hi[3], float rect[4]) {
    float x0 = 3.402823466e+38f, x1 = -3.402823466e+38f, y0 = 3.402823466e+38f, y1 = -3.402823466e+38f;
    v3 pos = V(c[0], c[1], c[2]), right = V(c[3], c[4], c[5]), up = V(c[6], c[7], c[8]), back = V(c[9], c[10], c[11]);
    for (int k = 0; k < 8; ++k) {
        v3 v = V(((k & 1) ? hi[0] : lo[0]) - pos.x, ((k & 2) ? hi[1] : lo[1]) - pos.y,
                 ((k & 4) ? hi[2] : lo[2]) - pos.z);
        float depth = -vdot(v, back);
        if (!(depth > 1.0e-4f)) return 0;
        float sx = vdot(v, right) / depth;
        float sy = vdot(v, up) / depth;
        float fx = (sx / c[12] + 1.0f) * (W * 0.5f);
        float fy = (1.0f - sy / c[13]) * (H * 0.5f);
        x0 = fminf(x0, fx); x1 = fmaxf(x1, fx);
        y0 = fminf(y0, fy); y1 = fmaxf(y1, fy);
    }
    rect[0] = x0 - 1.0f; rect[1] = x1 + 1.0f; rect[2] = y0 - 1.0f; rect[3] = y1 + 1.0f;
    return 1;
}

static mat_t load_mat(const float* mats, int id) {
    const float* m = mats + 12 * id;
    mat_t r;
    r.base = V(m[0], m[1], m[2]);
    r.metallic = m[3]; r.specular = m[4]; r.roughness = m[5]; r.ior = m[6];
    r.emission = V(m[7], m[8], m[9]);
    r.model = (int)m[10];
    return r;
}

/* Ray statistics of the last orc_render (orc_ray_counts): continuations and
 * shadow rays created at bounce 0 / at later bounces, as rr_frame_stats counts
 * them, and the first (pixel, sample) pairs whose path continued past bounce 1. */
/* Hull flags of an LDS-resident scene's triangle (csrc/wavefront.hip
 * stage_scene, hull_flags; same float operations): bit 0 when every vertex of
 * every triangle lies behind the triangle's plane on its front side (the
 * cross(e1, e2) direction, e1 = v1 - v0, e2 = v2 - v0), up to 2^-12 of the
 * vertex's distance times |n|_1,
 * bit 1 the same for the back side. A ray that leaves the triangle on a side
 * whose bit is set moves away from a plane the whole scene lies behind, so it
 * meets nothing: the continuation misses and the shadow ray is unoccluded
 * without a traversal (the skipped tests could only report rounding-level
 * grazing hits). */
static unsigned tri_hull(const lbvh* B, int i) {
    const float* s = B->tri + 9 * (size_t)i;
    const v3 v0 = V(s[0], s[1], s[2]);
    const v3 n = vcross(vsub(V(s[3], s[4], s[5]), v0), vsub(V(s[6], s[7], s[8]), v0));
    const float an = fabsf(n.x) + fabsf(n.y) + fabsf(n.z);
    int front = 1, back = 1;
    for (int j = 0; j < B->n; ++j) {
        const float* e = B->tri + 9 * (size_t)j;
        const v3 w[3] = {V(e[0], e[1], e[2]), V(e[3], e[4], e[5]), V(e[6], e[7], e[8])};
        for (int k = 0; k < 3; ++k) {
            const v3 r = vsub(w[k], v0);
            const float h = vdot(n, r);
            const float lim = an * (fabsf(r.x) + fabsf(r.y) + fabsf(r.z)) * 0x1p-12f;
            front = front && h <= lim;
            back = back && -h <= lim;
        }
    }
    return (unsigned)front | (unsigned)back << 1;
}

static long long g_rays[4];
/* wall seconds of the last orc_render's hierarchy build (orc_last_build_seconds):
 * the CPU baseline counts one build per frame, not one per rendered band */
static double g_build_s;
static double wall_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static int g_late[32], g_n_late;

/* The camera ray of (pix, sample) (csrc/wavefront.hip camera_ray_xy): the
 * subpixel pair is the 16-bit halves of the path key itself (a hash output),
 * filter-importance sampled; (fx, fy) its subpixel position. */
static void camera_ray(const scene_t* S, int pix, int sample, uint32_t* key_out, v3* o, v3* d, float* tmin,
                       float* tmax, float* fx_out, float* fy_out) {
    const float* c = S->cam;
    uint32_t key = pkey(S->seed, (uint32_t)pix, (uint32_t)sample);
    int px = pix % S->W, py = pix / S->W;
    const float ux = (float)(key >> 16) * 1.52587890625e-05f, uy = (float)(key & 0xffffu) * 1.52587890625e-05f;
    float fx = (float)px + 0.5f + lerp_table(S->filter, ORC_FILTER_N, ux);
    float fy = (float)py + 0.5f + lerp_table(S->filter, ORC_FILTER_N, uy);
    float sx = fmaf(fx, S->inv_w2, -1.0f) * c[12];
    float sy = fmaf(-fy, S->inv_h2, 1.0f) * c[13];
    float len = sqrtf(fmaf(sy, sy, fmaf(sx, sx, 1.0f)));
    v3 dw = V(fmaf(c[6], sy, fmaf(c[3], sx, -c[9])), fmaf(c[7], sy, fmaf(c[4], sx, -c[10])),
              fmaf(c[8], sy, fmaf(c[5], sx, -c[11])));
    float il = 1.0f / len;
    *d = vscl(dw, il);
    *o = V(c[0], c[1], c[2]);
    *tmin = c[14] * len;
    *tmax = c[15] * len;
    *key_out = key;
    *fx_out = fx;
    *fy_out = fy;
}

static v3 radiance(const scene_t* S, int pix, int sample, long long rays[4]) {
    uint32_t key;
    v3 o, d;
    float tmin, tmax, fx, fy;
    camera_ray(S, pix, sample, &key, &o, &d, &tmin, &tmax, &fx, &fy);
    v3 L = V(0.0f, 0.0f, 0.0f), T = V(1.0f, 1.0f, 1.0f);
    int nd = 0, ng = 0;  /* diffuse / glossy scatters so far (Cycles path_state_next) */
    int esc = 0;         /* the ray leaves a hull side of its triangle (tri_hull): it meets nothing */
    const int culled = S->cull_on && (fx < S->cull[0] || fx > S->cull[1] || fy < S->cull[2] || fy > S->cull[3]);
    for (int b = 0; b <= S->max_bounces; ++b) {
        hitrec h;
        if (b == 0 && culled) {
            h.t = tmax; h.u = h.v = 0.0f; h.idx = -1; h.orig = -1;
        } else if (b == 0 && S->cam_all) {
            /* wavefront.hip camera_hit: LDS-resident scenes test camera rays
             * against every triangle (the GPU bins them per 8x8 tile, which by
             * construction keeps every triangle a ray can hit; the accept rule
             * is order-independent, so the result is the same) */
            h.t = tmax; h.u = h.v = 0.0f; h.idx = -1; h.orig = -1;
            const shear_t sh = make_shear(d);
            for (int i = 0; i < S->bvh->n; ++i) try_leaf(S->bvh, i, &sh, o, tmin, &h);
        } else if (esc) {
            h.t = tmax; h.u = h.v = 0.0f; h.idx = -1; h.orig = -1;
        } else {
            trace(S->bvh, o, d, tmin, tmax, 0, &h);
        }
        if (h.idx < 0) {
            v3 cc = vmul(T, S->world);
            if (b > 0) cc = clampc(cc, S->clamp);
            L = vadd(L, cc);
            break;
        }
        const float* tp = S->bvh->tri + 9 * (size_t)h.idx;
        v3 e1 = vsub(V(tp[3], tp[4], tp[5]), V(tp[0], tp[1], tp[2])), e2 = vsub(V(tp[6], tp[7], tp[8]), V(tp[0], tp[1], tp[2]));
        const int mid = S->bvh->tri_mat[h.idx];
        mat_t m = load_mat(S->mats, mid);
        const float* lut = S->luts + ORC_LUT_STRIDE * (size_t)mid;
        float t = h.t;
        v3 P = vmadd(o, d, t);
        v3 N = vnorm(vcross(e1, e2));
        const int flip = vdot(N, d) > 0.0f;
        if (flip) N = V(-N.x, -N.y, -N.z);
        /* rays leaving this point go to N's side: the front side unless flipped */
        const int leave_esc = S->hull ? (int)((S->hull[h.idx] >> flip) & 1u) : 0;
        v3 wo = V(-d.x, -d.y, -d.z);
        if (m.emission.x != 0.0f || m.emission.y != 0.0f || m.emission.z != 0.0f) {
            v3 cc = vmul(T, m.emission);
            if (b > 0) cc = clampc(cc, S->clamp);
            L = vadd(L, cc);
        }
        /* Cycles path_state_next: the scatter that takes bounce, diffuse_bounce or
         * glossy_bounce to its cap ends the path at the next hit (emission only) */
        if (b >= S->max_bounces || nd >= S->max_diffuse || ng >= S->max_glossy) break;
        uint32_t dim0 = 2u + 8u * (uint32_t)b;
        /* dimension pairs of this bounce: (light pick, lobe choice) at dim0,
         * the disk point at dim0 + 1, the BSDF direction at dim0 + 4; the
         * Russian-roulette test keeps its own dimension dim0 + 6 */
        float u_light, u_lobe;
        rnd2(key, dim0, &u_light, &u_lobe);
        v3 Po = offset_ray(P, N);
        int shadow = 0;
        v3 sh_dir = V(0, 0, 0), sh_c = V(0, 0, 0);
        float sh_dist = 0.0f;
        if (S->n_lights > 0) {
            int li = (int)(u_light * (float)S->n_lights);
            if (li > S->n_lights - 1) li = S->n_lights - 1;
            const float* lt = S->lights + 12 * li;
            v3 wi, Li;
            float dist;
            if (lt[0] == 0.0f) {
                v3 lp = V(lt[1], lt[2], lt[3]);
                float radius = lt[7];
                v3 I = V(lt[8], lt[9], lt[10]);
                v3 tl = vsub(lp, P);
                float dl2 = vdot(tl, tl);
                if (radius > 0.0f) {
                    v3 wl = vscl(tl, 1.0f / sqrtf(dl2));
                    v3 b1, b2;
                    onb(wl, &b1, &b2);
                    float dx, dy;
                    float u1, u2;
                    rnd2(key, dim0 + 1u, &u1, &u2);
                    disk(u1, u2, &dx, &dy);
                    dx = dx * radius;
                    dy = dy * radius;
                    v3 sp = vmadd(vmadd(lp, b1, dx), b2, dy);
                    v3 ts = vsub(sp, P);
                    float ds2 = vdot(ts, ts);
                    dist = sqrtf(ds2);
                    float id = 1.0f / dist;
                    wi = vscl(ts, id);
                    float cl = fabsf(vdot(wl, wi));
                    Li = vscl(I, cl * id * id);
                } else {
                    dist = sqrtf(dl2);
                    wi = vscl(tl, 1.0f / dist);
                    Li = vscl(I, 1.0f / dl2);
                }
            } else {
                wi = V(-lt[4], -lt[5], -lt[6]);
                dist = 3.402823466e+38f;
                Li = V(lt[8], lt[9], lt[10]);
            }
            float cosN = vdot(N, wi);
            if (cosN > 0.0f) {
                float pdf;
                float ps = p_spec(lut, vdot(N, wo));
                v3 f = eval_bsdf(&m, lut, N, wo, wi, ps, &pdf); /* f * cosN */
                float k = (float)S->n_lights;
                v3 cc = V(T.x * f.x * k * Li.x, T.y * f.y * k * Li.y, T.z * f.z * k * Li.z);
                if (b > 0) cc = clampc(cc, S->clamp);
                if (vmax3(cc) > 0.0f) { shadow = 1; sh_dir = wi; sh_dist = dist; sh_c = cc; }
            }
        }
        int alive = 0, glossy = 0;
        v3 wi, f;
        float pdf;
        float u_b1, u_b2;
        rnd2(key, dim0 + 4u, &u_b1, &u_b2);
        if (sample_bsdf(&m, lut, N, wo, u_lobe, u_b1, u_b2, &wi, &f,
                        &pdf, &glossy)) {
            float k = 1.0f / pdf; /* f = f * cosL */
            T = V(T.x * f.x * k, T.y * f.y * k, T.z * f.z * k);
            alive = vmax3(T) > 0.0f;
            if (alive && b >= 3) {
                float q = fminf(vmax3(T), 1.0f);
                if (rnd(key, dim0 + 6u) >= q) alive = 0;
                else {
                    float iq = 1.0f / q;
                    T = V(T.x * iq, T.y * iq, T.z * iq);
                }
            }
        }
        {
            const int kb = b == 0 ? 0 : 2;
            rays[kb] += alive;  /* per row, summed after the row (orc_render) */
            rays[kb + 1] += shadow;
            if (b > 0 && alive) {
#pragma omp critical(orc_late)
                if (g_n_late < 16) { g_late[2 * g_n_late] = pix; g_late[2 * g_n_late + 1] = sample; ++g_n_late; }
            }
        }
        if (shadow) {
            hitrec hs;
            if (leave_esc || !trace(S->bvh, Po, sh_dir, 0.0f, sh_dist, 1, &hs)) L = vadd(L, sh_c);
        }
        if (!alive) break;
        if (glossy) ++ng; else ++nd;
        o = Po; d = wi; tmin = 0.0f; tmax = 3.402823466e+38f;
        esc = leave_esc;
    }
    return L;
}

/* ----------------------------------------------------- Filmic (view) ---- */
/* Blender 3.6's "Filmic" view for display sRGB, look None, as its OCIO config
 * chains it (restated in csrc/view.hpp): lg2 allocation [-12.473931188,
 * 12.526068812] -> filmic_desat65cube.spi3d (tetrahedral) -> uniform
 * allocation [0, 0.66] -> filmic_to_0-70_1-03.spi1d (linear). The LUT arrays
 * come from the caller (orc_set_filmic), parsed by oracle/host_oracle.py's own
 * .spi3d/.spi1d readers. Same float operations as csrc/view.hip. */
static struct {
    const float* cube; int n3;            /* n3^3 x rgb, entry (i, j, k) at (i n3 + j) n3 + k */
    const float* lut1; int n1, comps;     /* n1 x comps */
    float lo1, hi1;
} g_filmic;

void orc_set_filmic(const float* cube, int n3, const float* lut1, int n1, int comps, float lo1, float hi1) {
    g_filmic.cube = cube; g_filmic.n3 = n3;
    g_filmic.lut1 = lut1; g_filmic.n1 = n1; g_filmic.comps = comps;
    g_filmic.lo1 = lo1; g_filmic.hi1 = hi1;
}

/* log2 of a normal positive float without libm (csrc/view.hip log2_fixed) */
static float log2_fixed(float x) {
    int bits = fbits(x);
    int e = ((bits >> 23) & 0xff) - 127;
    float m = ibits((bits & 0x007fffff) | 0x3f800000);
    if (m > 1.41421356f) { m = m * 0.5f; e = e + 1; }
    float t = (m - 1.0f) / (m + 1.0f);
    float t2 = t * t;
    float p = ((((t2 * 0.111111112f + 0.142857149f) * t2 + 0.2f) * t2 + 0.333333343f) * t2 + 1.0f) * t;
    return (float)e + p * 2.88539004f;
}

static float lut1d(float x, int c) {
    const float* t = g_filmic.lut1;
    int n = g_filmic.n1, comps = g_filmic.comps;
    float f = (x - g_filmic.lo1) / (g_filmic.hi1 - g_filmic.lo1) * (float)(n - 1);
    f = fminf(fmaxf(f, 0.0f), (float)(n - 1));
    int i = (int)f;
    if (i >= n - 1) return t[(n - 1) * comps + c];
    float fr = f - (float)i;
    float a = t[i * comps + c], b = t[(i + 1) * comps + c];
    return a + (b - a) * fr;
}

static v3 cube_at(int i, int j, int k) {
    int n = g_filmic.n3;
    const float* q = g_filmic.cube + 3 * (((size_t)i * n + j) * n + k);
    return V(q[0], q[1], q[2]);
}

/* OCIO Lut3D tetrahedral interpolation, input clamped to [0, 1] */
static v3 lut3d_tetra(float r, float g, float b) {
    int n = g_filmic.n3;
    float s = (float)(n - 1);
    float fr = sat1(r) * s, fg = sat1(g) * s, fb = sat1(b) * s;
    int ir = (int)fr, ig = (int)fg, ib = (int)fb;
    if (ir > n - 2) ir = n - 2;
    if (ig > n - 2) ig = n - 2;
    if (ib > n - 2) ib = n - 2;
    fr = fr - (float)ir; fg = fg - (float)ig; fb = fb - (float)ib;
    v3 c000 = cube_at(ir, ig, ib), c111 = cube_at(ir + 1, ig + 1, ib + 1), c1, c2;
    float w0, w1, w2, w3;
    if (fr > fg) {
        if (fg > fb) { c1 = cube_at(ir + 1, ig, ib); c2 = cube_at(ir + 1, ig + 1, ib); w0 = 1.0f - fr; w1 = fr - fg; w2 = fg - fb; w3 = fb; }
        else if (fr > fb) { c1 = cube_at(ir + 1, ig, ib); c2 = cube_at(ir + 1, ig, ib + 1); w0 = 1.0f - fr; w1 = fr - fb; w2 = fb - fg; w3 = fg; }
        else { c1 = cube_at(ir, ig, ib + 1); c2 = cube_at(ir + 1, ig, ib + 1); w0 = 1.0f - fb; w1 = fb - fr; w2 = fr - fg; w3 = fg; }
    } else {
        if (fb > fg) { c1 = cube_at(ir, ig, ib + 1); c2 = cube_at(ir, ig + 1, ib + 1); w0 = 1.0f - fb; w1 = fb - fg; w2 = fg - fr; w3 = fr; }
        else if (fb > fr) { c1 = cube_at(ir, ig + 1, ib); c2 = cube_at(ir, ig + 1, ib + 1); w0 = 1.0f - fg; w1 = fg - fb; w2 = fb - fr; w3 = fr; }
        else { c1 = cube_at(ir, ig + 1, ib); c2 = cube_at(ir + 1, ig + 1, ib); w0 = 1.0f - fg; w1 = fg - fr; w2 = fr - fb; w3 = fb; }
    }
    return V(((w0 * c000.x + w1 * c1.x) + w2 * c2.x) + w3 * c111.x,
             ((w0 * c000.y + w1 * c1.y) + w2 * c2.y) + w3 * c111.y,
             ((w0 * c000.z + w1 * c1.z) + w2 * c2.z) + w3 * c111.z);
}

static unsigned char q8(float f);

static void filmic8(const float c[3], unsigned char* out) {
    float a[3];
    for (int k = 0; k < 3; ++k) a[k] = (log2_fixed(fmaxf(c[k], 1.17549435e-38f)) + 12.473931188f) / 25.0f;
    v3 b = lut3d_tetra(a[0], a[1], a[2]);
    float bb[3] = {b.x, b.y, b.z};
    for (int k = 0; k < 3; ++k) out[k] = q8(lut1d(bb[k] / 0.66f, g_filmic.comps == 3 ? k : 0));
}

/* Filmic of n linear RGB triples (tests of the chain in isolation) */
void orc_filmic(int n, const float* rgb, unsigned char* out3) {
    for (int i = 0; i < n; ++i) filmic8(rgb + 3 * (size_t)i, out3 + 3 * (size_t)i);
}

static unsigned char q8(float f) {
    if (f <= 0.0f) return 0;
    if (f >= 1.0f) return 255;
    return (unsigned char)(f * 255.0f + 0.5f);
}

/* ------------------------------------------------------------ C entry ---- */

int orc_abi(void) { return 2; }

/* LBVH of n triangles (tris9: v0 v1 v2 per triangle). Outputs as rr_debug_bvh. */
int orc_build_bvh(int n, const float* tris9, int hier, uint32_t* keys, uint32_t* order, int32_t* children,
                  float* boxes) {
    lbvh B;
    lbvh_build(&B, n, tris9, NULL, hier);
    if (n > 0) {
        int ni = n > 1 ? n - 1 : 1;
        if (keys) memcpy(keys, B.keys, sizeof(uint32_t) * n);
        if (order) memcpy(order, B.order, sizeof(uint32_t) * n);
        if (children) memcpy(children, B.child_lf, sizeof(int32_t) * 2 * ni);
        if (boxes) memcpy(boxes, B.box, sizeof(float) * 12 * ni);
    }
    lbvh_free(&B);
    return 0;
}

int orc_build_lbvh(int n, const float* tris9, uint32_t* keys, uint32_t* order, int32_t* children, float* boxes) {
    return orc_build_bvh(n, tris9, 2, keys, order, children, boxes);
}

/* Brute force closest hit (no BVH), for pinning the LBVH traversal. */
int orc_trace_brute(int n, const float* tris9, int n_rays, const float* rays, float* hits, int32_t* prims) {
    for (int r = 0; r < n_rays; ++r) {
        const float* R = rays + 8 * (size_t)r;
        v3 o = V(R[0], R[1], R[2]), d = V(R[4], R[5], R[6]);
        const shear_t sh = make_shear(d);
        float best = R[7];
        int bo = -1;
        float bu = 0, bv = 0;
        for (int i = 0; i < n; ++i) {
            float tt, u, v;
            if (!woop_test(&sh, o, tris9 + 9 * (size_t)i, &tt, &u, &v)) continue;
            if (tt > R[3] && (tt < best || (tt == best && i < bo))) { best = tt; bo = i; bu = u; bv = v; }
        }
        if (hits) { hits[4 * r] = bo >= 0 ? best : R[7]; hits[4 * r + 1] = bu; hits[4 * r + 2] = bv; hits[4 * r + 3] = 0; }
        if (prims) prims[r] = bo;
    }
    return 0;
}

/* Quantised wide BVH (rr_debug_bvh4 layout): n4 nodes, ORC_QW_MAX child refs and the 16
 * words of each node. */
int orc_build_qbvh(int n, const float* tris9, int32_t* n4, int32_t* children4, uint32_t* nodes16,
                   int32_t* tri_orig) {
    lbvh B;
    lbvh_build(&B, n, tris9, NULL, 3);
    lbvh_collapse4(&B);
    *n4 = B.n4;
    if (children4 && B.n4) memcpy(children4, B.child4, sizeof(int32_t) * ORC_QW_MAX * (size_t)B.n4);
    if (nodes16 && B.n4) memcpy(nodes16, B.q4, sizeof(uint32_t) * 16 * (size_t)B.n4);
    if (tri_orig && n > 0) memcpy(tri_orig, B.tri_orig, sizeof(int32_t) * (size_t)n);
    lbvh_free(&B);
    return 0;
}

int orc_trace_w(int n, const float* tris9, int width, int n_rays, const float* rays, float* hits, int32_t* prims,
                uint8_t* occluded) {
    lbvh B;
    lbvh_build(&B, n, tris9, NULL, width == 4 ? 3 : width);
    if (width == 4) { lbvh_collapse4(&B); B.width = 4; }
    for (int r = 0; r < n_rays; ++r) {
        const float* R = rays + 8 * (size_t)r;
        v3 o = V(R[0], R[1], R[2]), d = V(R[4], R[5], R[6]);
        hitrec h, h2;
        trace(&B, o, d, R[3], R[7], 0, &h);
        if (hits) { hits[4 * r] = h.t; hits[4 * r + 1] = h.u; hits[4 * r + 2] = h.v; hits[4 * r + 3] = 0.0f; }
        if (prims) prims[r] = h.orig;
        if (occluded) occluded[r] = (uint8_t)trace(&B, o, d, R[3], R[7], 1, &h2);
    }
    lbvh_free(&B);
    return 0;
}

#ifdef ORC_WALK_STUDY
/* Research build only (tools/beam_study.py): the device's any-hit beam packet
 * walk (packet_shadow_beam of commit 76f0210) over packets of rays starts[k] ..
 * starts[k + 1] - 1 (at most 64; 8 floats each: o, tmin, d, tmax), against
 * the per-lane any-hit walk.
 * out: [0] packets, [1] beam node visits (per packet), [2] beam leaf tests
 * (summed over lanes), [3] per-lane node visits, [4] per-lane leaf tests,
 * [5] rays whose occlusion differs, [6] blocked rays. */
static float st_min(const float* v, int n, int mx) {
    float r = mx ? -INFINITY : INFINITY;
    for (int i = 0; i < n; ++i) r = mx ? fmaxf(r, v[i]) : fminf(r, v[i]);
    return r;
}
int orc_study_beam(int n, const float* tris9, int n_packets, const int* starts, const float* rays, long long* out) {
    lbvh B;
    lbvh_build(&B, n, tris9, NULL, 3);
    lbvh_collapse4(&B);
    B.width = 4;
    for (int k = 0; k < 7; ++k) out[k] = 0;
    for (int pk = 0; pk < n_packets; ++pk) {
        const int p0 = starts[pk];
        const int m = starts[pk + 1] - p0 < 64 ? starts[pk + 1] - p0 : 64;
        if (m <= 0) continue;
        float ox[64], oy[64], oz[64], ix[64], iy[64], iz[64], dx[64], dy[64], dz[64], tm[64];
        shear_t sh[64];
        hitrec h[64];
        int live[64], occ_ref[64];
        for (int i = 0; i < m; ++i) {
            const float* R = rays + 8 * (size_t)(p0 + i);
            v3 o = V(R[0], R[1], R[2]), d = V(R[4], R[5], R[6]);
            v3 iq = rcp3(d);
            ox[i] = o.x; oy[i] = o.y; oz[i] = o.z; dx[i] = d.x; dy[i] = d.y; dz[i] = d.z;
            ix[i] = iq.x; iy[i] = iq.y; iz[i] = iq.z; tm[i] = R[7];
            sh[i] = make_shear(d);
            h[i].t = R[7]; h[i].u = h[i].v = 0.0f; h[i].idx = -1; h[i].orig = -1;
            live[i] = 1;
            long long save[6];
            orc_walk_counts(save, 1);
            hitrec hr;
            occ_ref[i] = trace4(&B, o, d, 0.0f, R[7], 1, &hr);
            long long c6[6];
            orc_walk_counts(c6, 1);
            out[3] += c6[0]; out[4] += c6[1];
        }
        const float ol[3] = {st_min(ox, m, 0), st_min(oy, m, 0), st_min(oz, m, 0)};
        const float oh[3] = {st_min(ox, m, 1), st_min(oy, m, 1), st_min(oz, m, 1)};
        const float il[3] = {st_min(ix, m, 0), st_min(iy, m, 0), st_min(iz, m, 0)};
        const float ih[3] = {st_min(ix, m, 1), st_min(iy, m, 1), st_min(iz, m, 1)};
        const float dl[3] = {st_min(dx, m, 0), st_min(dy, m, 0), st_min(dz, m, 0)};
        const float dh[3] = {st_min(dx, m, 1), st_min(dy, m, 1), st_min(dz, m, 1)};
        const float t_hi = st_min(tm, m, 1);
        int stack[4096], sp = 0, node = 0, n_live = m;
        ++out[0];
        for (;;) {
            ++out[1];
            const uint32_t* nd = B.q4 + 16 * (size_t)node;
            const uint32_t inner = nd[3] >> 24;
            float org[3];
            memcpy(org, nd, sizeof org);
            float mo = 0.0f;
            for (int a = 0; a < 3; ++a) mo = fmaxf(mo, fmaxf(fabsf(org[a] - oh[a]), fabsf(org[a] - ol[a])));
            const float m2 = 2.0f * fmaf(mo, ORC_BOX_MARGIN, ldexpf(255.0f * ORC_BOX_MARGIN, (int)((nd[15] >> 8) & 255u) - 128));
            float tn[ORC_QW_MAX];
            int pass[ORC_QW_MAX];
            for (int c = 0; c < ORC_QW_MAX; ++c) {
                float nr3[3], fr3[3];
                for (int a = 0; a < 3; ++a) {
                    const int e = (int)((nd[3] >> (8 * a)) & 255u) - 128;
                    uint32_t ql, qh;
                    if (c < 4) { ql = (nd[6 + a] >> (8 * c)) & 255u; qh = (nd[9 + a] >> (8 * c)) & 255u; }
                    else {
                        const uint32_t lo2 = (nd[12 + a / 2] >> (16 * (a & 1))) & 0xffffu;
                        const uint32_t hi2 = (nd[12 + (3 + a) / 2] >> (16 * ((3 + a) & 1))) & 0xffffu;
                        ql = (lo2 >> (8 * (c - 4))) & 255u; qh = (hi2 >> (8 * (c - 4))) & 255u;
                    }
                    const float lo = (org[a] - oh[a]) + ldexpf((float)ql, e) - m2;
                    const float hi = (org[a] - ol[a]) + ldexpf((float)qh, e) + m2;
                    float nr, fr;
                    if (il[a] > 0.0f) { nr = lo * (lo >= 0.0f ? il[a] : ih[a]); fr = hi * (hi >= 0.0f ? ih[a] : il[a]); }
                    else if (ih[a] < 0.0f) { nr = hi * (hi >= 0.0f ? il[a] : ih[a]); fr = lo * (lo >= 0.0f ? ih[a] : il[a]); }
                    else {
                        fr = INFINITY; nr = 0.0f;
                        if (lo > 0.0f) nr = dh[a] > 0.0f ? lo / dh[a] : INFINITY;
                        if (hi < 0.0f) nr = dl[a] < 0.0f ? hi / dl[a] : INFINITY;
                    }
                    nr3[a] = nr; fr3[a] = fr;
                }
                tn[c] = fmaxf(fmaxf(nr3[0], nr3[1]), fmaxf(nr3[2], 0.0f));
                const float tf = fminf(fminf(fr3[0], fr3[1]), fminf(fr3[2], t_hi));
                pass[c] = tn[c] <= tf && ((nd[15] >> c) & 1u);
            }
            int n_lf = 0, n_in = 0, best = -1;
            for (int c = 0; c < ORC_QW_MAX; ++c) {
                const int is_inner = (inner >> c) & 1u;
                if (!is_inner) {
                    if (pass[c]) {
                        const int ti = (int)nd[5] + n_lf;
                        for (int i = 0; i < m; ++i) {
                            if (!live[i]) continue;
                            ++out[2];
                            try_leaf(&B, ti, &sh[i], V(ox[i], oy[i], oz[i]), 0.0f, &h[i]);
                            if (h[i].idx >= 0) { live[i] = 0; --n_live; }
                        }
                    }
                    ++n_lf;
                } else {
                    if (pass[c] && (best < 0 || tn[c] < tn[best])) best = c;
                    ++n_in;
                }
            }
            if (n_live == 0) break;
            if (best < 0) {
                if (sp == 0) break;
                node = stack[--sp];
                continue;
            }
            for (int c = ORC_QW_MAX - 1, rank; c >= 0; --c) {
                if (!((inner >> c) & 1u) || c == best || !pass[c]) continue;
                rank = 0;
                for (int q = 0; q < c; ++q) rank += (inner >> q) & 1u;
                if (sp < 4096) stack[sp++] = (int)nd[4] + rank;
            }
            int rb = 0;
            for (int q = 0; q < best; ++q) rb += (inner >> q) & 1u;
            node = (int)nd[4] + rb;
        }
        for (int i = 0; i < m; ++i) {
            const int occ = h[i].idx >= 0;
            out[5] += occ != occ_ref[i];
            out[6] += occ;
        }
    }
    lbvh_free(&B);
    return 0;
}
#endif

int orc_trace(int n, const float* tris9, int n_rays, const float* rays, float* hits, int32_t* prims,
              uint8_t* occluded) {
    return orc_trace_w(n, tris9, 2, n_rays, rays, hits, prims, occluded);
}

/* Full frame. render_ints: W H spp max_bounces seed view_transform (as rr.h);
 * render_floats: clamp_indirect filter_width exposure_scale.
 * film: W*H*4 floats of mean radiance; rgba8: W*H*4 bytes. Rows
 * [row_begin, row_end) only (row_end <= 0: all rows), so a bounded sample of a
 * frame can be timed. threads <= 0: OpenMP default. */
#define ORC_FILM_GROUP 32

double orc_last_build_seconds(void) { return g_build_s; }

/* The two shortcuts orc_render shares with the product, switchable so the
 * tests can show that neither changes a pixel (tests/test_oracle.py):
 *  cull: camera rays outside the scene's screen rectangle (screen_rect) are
 *        misses without a traversal (csrc/wavefront.hip camera_ray_xy);
 *  hull: on LDS-resident scenes (render_ints[7] == 2) a secondary ray leaving
 *        a hull side of its triangle (tri_hull) is a miss / unoccluded without
 *        a traversal (csrc/wavefront.hip hull_flags).
 * Both are on by default (what the product does). */
static int g_rule_cull = 1, g_rule_hull = 1;
void orc_set_rules(int cull, int hull) { g_rule_cull = cull; g_rule_hull = hull; }

void orc_ray_counts(long long* out4, int* late32, int* n_late) {
    for (int k = 0; k < 4; ++k) out4[k] = g_rays[k];
    for (int k = 0; k < 2 * g_n_late; ++k) late32[k] = g_late[k];
    *n_late = g_n_late;
}

/* rows rendered by the next orc_render calls instead of [row_begin, row_end)
 * (NULL: the range): spread sample rows of a large frame with one hierarchy
 * build (test use; orc_set_row_list(NULL, 0) resets) */
static const int32_t* g_row_list;
static int g_n_row_list;
void orc_set_row_list(const int32_t* rows, int n) { g_row_list = n > 0 ? rows : NULL; g_n_row_list = n > 0 ? n : 0; }

int orc_render(int n_tris, const float* tris9, const int32_t* tri_mat, const float* cam, int n_lights,
               const float* lights, const float* mats, const float* world, const int32_t* ri, const float* rf,
               float* film, uint8_t* rgba8, int row_begin, int row_end, int threads) {
    memset(g_rays, 0, sizeof g_rays);
    g_n_late = 0;
    lbvh B;
    const double t_build = wall_s();
    lbvh_build(&B, n_tris, tris9, tri_mat, (ri[7] == 3 || ri[7] == 4) ? 3 : 2);  /* the hierarchy the product walks */
    if (ri[7] == 4) { lbvh_collapse4(&B); B.width = 4; }
    g_build_s = wall_s() - t_build;
    scene_t* S = (scene_t*)calloc(1, sizeof(scene_t));
    S->bvh = &B;
    S->cam = cam;
    S->n_lights = n_lights;
    S->lights = lights;
    S->mats = mats;
    S->world = V(world[0], world[1], world[2]);
    S->cam_all = ri[7] == 2;
    if (S->cam_all && n_tris > 0 && g_rule_hull) {
        S->hull = (unsigned char*)malloc((size_t)n_tris);
        for (int i = 0; i < n_tris; ++i) S->hull[i] = (unsigned char)tri_hull(&B, i);
    }
    S->W = ri[0]; S->H = ri[1]; S->spp = ri[2]; S->max_bounces = ri[3]; S->seed = (uint32_t)ri[4]; S->view = ri[5];
    S->max_diffuse = ri[8]; S->max_glossy = ri[9];
    {
        int nm = 0; /* materials referenced by triangles (the product tables every scene material) */
        for (int i = 0; i < n_tris; ++i) if (tri_mat[i] + 1 > nm) nm = tri_mat[i] + 1;
        S->luts = (float*)calloc((size_t)(nm > 0 ? nm : 1) * ORC_LUT_STRIDE, sizeof(float));
        for (int i = 0; i < nm; ++i) orc_material_lut(mats + 12 * (size_t)i, S->luts + ORC_LUT_STRIDE * (size_t)i);
    }
    S->clamp = rf[0];
    S->inv_w2 = 2.0f / (float)S->W;
    S->inv_h2 = 2.0f / (float)S->H;
    orc_filter_table(rf[1], S->filter);
    orc_srgb_lut(S->srgb);
    if (n_tris > 0) {
        const float* r = B.box; /* root: two child boxes */
        float lo[3] = {fminf(r[0], r[6]), fminf(r[1], r[7]), fminf(r[2], r[8])};
        float hi[3] = {fmaxf(r[3], r[9]), fmaxf(r[4], r[10]), fmaxf(r[5], r[11])};
        S->cull_on = g_rule_cull ? screen_rect(cam, (float)S->W, (float)S->H, lo, hi, S->cull) : 0;
    }
    const float exposure = rf[2];
    const float inv_spp = 1.0f / (float)S->spp;
    if (row_end <= 0 || row_end > S->H) row_end = S->H;
    if (row_begin < 0) row_begin = 0;
    /* work items of ORC_SEG pixels of one row, so that a band of a few rows
     * still spreads over every thread (per-pixel results do not depend on the
     * split) */
    const int nseg = (S->W + ORC_SEG - 1) / ORC_SEG;
    const long n_items = (long)(g_row_list ? g_n_row_list : row_end - row_begin) * nseg;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (long it = 0; it < n_items; ++it) {
        const int y = g_row_list ? g_row_list[it / nseg] : row_begin + (int)(it / nseg);
        const int x0 = (int)(it % nseg) * ORC_SEG;
        const int x1 = x0 + ORC_SEG < S->W ? x0 + ORC_SEG : S->W;
        long long rays[4] = {0, 0, 0, 0};
        for (int x = x0; x < x1; ++x) {
            int pix = y * S->W + x;
            /* film sum order (the product's kFilmGroup, csrc/wavefront.hip): in
             * order within groups of ORC_FILM_GROUP samples, group sums in order */
            v3 acc = V(0.0f, 0.0f, 0.0f);
            for (int g0 = 0; g0 < S->spp; g0 += ORC_FILM_GROUP) {
                v3 P = V(0.0f, 0.0f, 0.0f);
                const int g1 = g0 + ORC_FILM_GROUP < S->spp ? g0 + ORC_FILM_GROUP : S->spp;
                for (int s = g0; s < g1; ++s) {
                    v3 L = radiance(S, pix, s, rays);
                    P.x = P.x + L.x;
                    P.y = P.y + L.y;
                    P.z = P.z + L.z;
                }
                acc.x = acc.x + P.x;
                acc.y = acc.y + P.y;
                acc.z = acc.z + P.z;
            }
            if (film) {
                film[4 * (size_t)pix] = acc.x * inv_spp;
                film[4 * (size_t)pix + 1] = acc.y * inv_spp;
                film[4 * (size_t)pix + 2] = acc.z * inv_spp;
                film[4 * (size_t)pix + 3] = 1.0f;
            }
            if (rgba8 && S->view == 2) {
                float c3[3] = {acc.x * inv_spp * exposure, acc.y * inv_spp * exposure, acc.z * inv_spp * exposure};
                filmic8(c3, rgba8 + 4 * (size_t)pix);
                rgba8[4 * (size_t)pix + 3] = 255;
            } else if (rgba8) {
                float c3[3] = {acc.x * inv_spp * exposure, acc.y * inv_spp * exposure, acc.z * inv_spp * exposure};
                for (int k = 0; k < 3; ++k) {
                    float v = fminf(fmaxf(c3[k], 0.0f), 1.0f);
                    if (S->view == 0) v = v <= 0.0031308f ? v * 12.92f : lerp_table(S->srgb, ORC_SRGB_N + 1, v);
                    rgba8[4 * (size_t)pix + k] = q8(v);
                }
                rgba8[4 * (size_t)pix + 3] = 255;
            }
        }
        for (int k = 0; k < 4; ++k) {
#pragma omp atomic
            g_rays[k] += rays[k];
        }
    }
    free(S->luts);
    free(S->hull);
    free(S);
    lbvh_free(&B);
    return 0;
}

/* Camera rays of (pixel, sample) pairs as rays of orc_trace (o, tmin, d,
 * tmax per ray), for the camera floats / render ints / render floats of
 * rr_debug_frame_state: tests trace the rays of individual paths. */
void orc_camera_rays(const float* cam, const int32_t* ri, const float* rf, int n, const int32_t* pix,
                     const int32_t* sample, float* rays8) {
    scene_t* S = (scene_t*)calloc(1, sizeof(scene_t));
    S->cam = cam;
    S->W = ri[0]; S->H = ri[1]; S->seed = (uint32_t)ri[4];
    S->inv_w2 = 2.0f / (float)S->W;
    S->inv_h2 = 2.0f / (float)S->H;
    orc_filter_table(rf[1], S->filter);
    for (int i = 0; i < n; ++i) {
        uint32_t key;
        v3 o, d;
        float tmin, tmax, fx, fy;
        camera_ray(S, pix[i], sample[i], &key, &o, &d, &tmin, &tmax, &fx, &fy);
        float* r = rays8 + 8 * (size_t)i;
        r[0] = o.x; r[1] = o.y; r[2] = o.z; r[3] = tmin;
        r[4] = d.x; r[5] = d.y; r[6] = d.z; r[7] = tmax;
    }
    free(S);
}

/* Expose a few primitives for the known-answer tests. */
void orc_rng(uint32_t seed, uint32_t pixel, uint32_t sample, int ndims, float* out) {
    uint32_t k = pkey(seed, pixel, sample);
    for (int i = 0; i < ndims; ++i) out[i] = rnd(k, (uint32_t)i);
}

void orc_disk(int n, const float* u, float* xy) {
    for (int i = 0; i < n; ++i) disk(u[2 * i], u[2 * i + 1], &xy[2 * i], &xy[2 * i + 1]);
}

/* BSDF sampling for the estimator tests (tests/test_oracle.py): n draws of
 * sample_bsdf at one shading point, u = n x (ul, u1, u2) -> wi (3), f (3),
 * pdf and ok per draw (ok = 0: the path ends, as in radiance()). */
/* exports report the BSDF value f = (f * cosL) / cosL */
static v3 f_of(v3 fcos, float cosL) { return cosL > 0.0f ? V(fcos.x / cosL, fcos.y / cosL, fcos.z / cosL) : fcos; }

void orc_bsdf_sample(const float* mat12, const float* n3, const float* wo3, int n, const float* u, float* wi3,
                     float* f3, float* pdf, int32_t* ok) {
    mat_t m = load_mat(mat12, 0);
    float lut[ORC_LUT_STRIDE];
    orc_material_lut(mat12, lut);
    v3 N = V(n3[0], n3[1], n3[2]), wo = V(wo3[0], wo3[1], wo3[2]);
    for (int i = 0; i < n; ++i) {
        v3 wi = V(0.0f, 0.0f, 0.0f), f = wi;
        float p = 0.0f;
        int glossy = 0;
        ok[i] = sample_bsdf(&m, lut, N, wo, u[3 * i], u[3 * i + 1], u[3 * i + 2], &wi, &f, &p, &glossy);
        if (ok[i]) {
            ok[i] = 1 + glossy;  /* 1 diffuse lobe, 2 glossy lobe (rr_debug_bsdf_sample) */
            f = f_of(f, vdot(N, wi));
        }
        wi3[3 * i] = wi.x; wi3[3 * i + 1] = wi.y; wi3[3 * i + 2] = wi.z;
        f3[3 * i] = f.x; f3[3 * i + 1] = f.y; f3[3 * i + 2] = f.z;
        pdf[i] = p;
    }
}

/* Batched BSDF eval at one shading point (estimator tests): n directions wi. */
void orc_bsdf_eval_n(const float* mat12, const float* n3, const float* wo3, int n, const float* wi3, float* f3,
                     float* pdf) {
    mat_t m = load_mat(mat12, 0);
    float lut[ORC_LUT_STRIDE];
    orc_material_lut(mat12, lut);
    v3 N = V(n3[0], n3[1], n3[2]), wo = V(wo3[0], wo3[1], wo3[2]);
    float ps = p_spec(lut, vdot(N, wo));
    for (int i = 0; i < n; ++i) {
        v3 wi = V(wi3[3 * i], wi3[3 * i + 1], wi3[3 * i + 2]);
        v3 f = f_of(eval_bsdf(&m, lut, N, wo, wi, ps, &pdf[i]), vdot(N, wi));
        f3[3 * i] = f.x; f3[3 * i + 1] = f.y; f3[3 * i + 2] = f.z;
    }
}

/* BSDF eval for known-answer tests: mat12, N, wo, wi -> f (3), pdf. */
void orc_bsdf_eval(const float* mat12, const float* n3, const float* wo3, const float* wi3, float* f3, float* pdf) {
    mat_t m = load_mat(mat12, 0);
    float lut[ORC_LUT_STRIDE];
    orc_material_lut(mat12, lut);
    v3 N = V(n3[0], n3[1], n3[2]), wo = V(wo3[0], wo3[1], wo3[2]), wi = V(wi3[0], wi3[1], wi3[2]);
    float ps = p_spec(lut, vdot(N, wo));
    v3 f = f_of(eval_bsdf(&m, lut, N, wo, wi, ps, pdf), vdot(N, wi));
    f3[0] = f.x; f3[1] = f.y; f3[2] = f.z;
}
