// Host-side interface of the device module: buffers in HBM and the launch
// sequences of the LBVH build (bvh.hip) and the wavefront integrator
// (wavefront.hip). DESIGN.md §4 describes the layout.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rr.h"
#include "rr_device.h"

namespace rr {

struct HipError : std::runtime_error {
    int code;
    HipError(const std::string& what, int c) : std::runtime_error(what), code(c) {}
};

#define RR_HIP(call)                                                                             \
    do {                                                                                         \
        hipError_t _e = (call);                                                                  \
        if (_e != hipSuccess)                                                                    \
            throw ::rr::HipError(std::string(#call) + ": " + hipGetErrorString(_e), (int)_e);   \
    } while (0)

// Grow-only device allocation.
template <typename T>
struct DevBuf {
    T* ptr = nullptr;
    size_t cap = 0;  // elements
    void ensure(size_t n) {
        if (n <= cap) return;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        if (n == 0) return;
        RR_HIP(hipMalloc(&ptr, n * sizeof(T)));
        cap = n;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// Per-scene geometry + acceleration structure.
struct DevScene {
    int n_tris = 0;
    int n_objs = 0;
    DevBuf<float4> tri_local;  // 3 per triangle, object space
    DevBuf<int32_t> tri_obj;
    DevBuf<int32_t> tri_mat;
    DevBuf<float> obj_xform;   // 12 per object
    DevBuf<float4> tri_world;  // 3 per triangle, world space (this frame)
    // LBVH build scratch
    DevBuf<uint32_t> bounds;    // 6 ordered-uint words (centroid-sum AABB)
    DevBuf<uint32_t> keys[2], vals[2];
    DevBuf<uint32_t> hist;      // 256 * nblocks
    DevBuf<uint32_t> scan_part; // partial sums of the scan
    DevBuf<int2> children;      // n-1
    DevBuf<int32_t> node_parent;  // n-1 : parent*2+side, -1 root
    DevBuf<int32_t> leaf_parent;  // n
    DevBuf<uint32_t> flags;       // n-1 arrival counters
    DevBuf<int2> range;           // n-1 : (first sorted leaf, leaf count) under each node
    // acceleration structure consumed by traversal
    DevBuf<BvhNode> nodes;  // max(n-1, 1)
    DevBuf<TriPack> tris;   // n, leaf order (after a BVH4 collapse: the BVH4's leaf order)
    DevBuf<QNode6> qnodes;     // quantised 6-wide collapse of `nodes` (split path), <= n-1
    DevBuf<float4> tnrm;       // split path, per triangle in leaf order: unit geometric normal, material id (shading)
    DevBuf<TriPack> qtris;     // collapse scratch: the triangles in the collapse's leaf order (swapped into `tris`)
    DevBuf<int32_t> q_src;     // wide node -> its BVH2 root (collapse scratch)
    DevBuf<uint32_t> q_cnt;    // per frontier node: internal children (scanned in place)
    DevBuf<uint32_t> q_tcnt;   // per frontier node: leaf children (scanned in place)
    DevBuf<int32_t> q_ctl;     // current level [lo, hi), first triangle of the level
    int nq = 0;                // wide nodes
    bool has4 = false;
    // PLOC build (large scenes): cluster ping-pong, neighbours, scan flags, counters
    DevBuf<float4> ploc_cl[2];
    DevBuf<int32_t> ploc_nn;
    DevBuf<uint32_t> ploc_keep, ploc_mrg;
    DevBuf<int32_t> ploc_ctl;
    bool ploc = false;  // the current nodes come from PLOC (else the Karras LBVH)
    std::vector<float> cached_xform;  // obj_xform of the current build
    bool built = false;
    bool uploaded = false;
    void release();
};

// Optional per-launch HIP-event timing (RR_FLAG_PROFILE_KERNELS), on the
// stream the kernels run on.
struct KernelProfiler {
    bool on = false;
    std::vector<hipEvent_t> pool;
    std::vector<int> cls;  // class of event pair i
    size_t used = 0;       // events in use (pairs * 2)
    void reset(bool enable) {
        on = enable;
        used = 0;
        cls.clear();
    }
    void begin(hipStream_t st, int c) {
        if (!on) return;
        while (pool.size() < used + 2) {
            hipEvent_t e;
            RR_HIP(hipEventCreate(&e));
            pool.push_back(e);
        }
        cls.push_back(c);
        RR_HIP(hipEventRecord(pool[used], st));
    }
    void end(hipStream_t st) {
        if (!on) return;
        RR_HIP(hipEventRecord(pool[used + 1], st));
        used += 2;
    }
    // after the stream has been synchronised
    void collect(double* ms, int32_t* launches) {
        for (size_t i = 0; i < cls.size(); ++i) {
            float t = 0.f;
            RR_HIP(hipEventElapsedTime(&t, pool[2 * i], pool[2 * i + 1]));
            ms[cls[i]] += t;
            launches[cls[i]] += 1;
        }
    }
    void release() {
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
        pool.clear();
    }
};

// Per-context wavefront state (sized for the largest chunk seen).
struct DevPaths {
    size_t cap = 0;
    DevBuf<float4> rad;                        // per path (p-indexed) radiance record
    DevBuf<float4> ps_o[2], ps_d[2], ps_t[2];  // segmented path queue, ping-pong per bounce
    DevBuf<float4> sh_o, sh_d, sh_c;           // segmented shadow queue
    DevBuf<float2> hits;                       // split path: (t, leaf index) per queue entry
    DevBuf<uint32_t> qctr;                     // split path: grouped queue append counters
    DevBuf<uint32_t> perm;                     // split path, RR_RAY_SORT: queue position -> slot (k_sort_queue)
    DevBuf<int32_t> counters;  // per chunk, per bounce b: {paths entering b+1, shadow rays of b}
    DevBuf<int32_t> spill;     // traversal stack spill
    DevBuf<float4> film;
    DevBuf<float4> film_part;  // open sample group's partial sum between chunks (k_accumulate)
    DevBuf<float> tile_slab;   // k_tiles: per sliced tile, one group sum plane per sample group
    DevBuf<uint32_t> tile_ctrs;  // k_tiles: work-unit counters, one 128-B line per shard
    DevBuf<uint32_t> tile_cost;  // k_tiles: per screen tile, the real-time ticks its units took (last launch)
    DevBuf<int32_t> tile_order;  // k_tiles: box tiles by descending tile_cost (k_tile_order)
    DevBuf<uint8_t> rgba8;
    DevBuf<float> filter_table;
    DevBuf<float> srgb_lut;
    DevBuf<float> lights, materials;
    DevBuf<float> mat_lut;             // material tables (build_material_lut), uploaded when they change
    std::vector<float> mat_lut_cached;
    DevBuf<unsigned long long> trav_counts;  // RR_FLAG_COUNT_TRAVERSAL: kTravWords
    KernelProfiler prof;
    bool count_traversal = false;
    bool force_wavefront = false;  // RR_FLAG_WAVEFRONT: LDS-resident scenes take the split path, not k_tiles
    bool tile_whole = false;       // k_tiles: one work unit per tile (the frame overlaps a pending one)
    int last_tile_slices = 0;      // render_frame_device: k_tiles units per box tile of the last frame (0: not k_tiles)
    bool last_unit_logged = false; // render_frame_device: the last k_tiles launch wrote its unit log (trav_counts)
    int grid_blocks = 0;  // persistent grid for path kernels
    void ensure_paths(size_t n);
    void ensure_tiles();  // k_tiles: only the traversal stack spill area
    void release();
};

// Frame constants passed by value to the path kernels.
struct FrameConsts {
    float3 cam_pos, cam_right, cam_up, cam_back;
    float half_w, half_h, clip_start, clip_end;
    float inv_w2, inv_h2;  // 2/W, 2/H
    int W, H, npix;
    // pixel index -> (x, y); split-path index p = pixel * spp_chunk + sample ->
    // (pixel, sample): pixel-major, so the samples of a pixel are neighbours in
    // every per-path array (set per chunk, render_split)
    FastDiv div_w, div_spp;
    int spp_total, spp_chunk, first_sample, max_bounces, n_lights;
    int max_diffuse, max_glossy;  // per-lobe bounce caps (>= 1, setup_frame)
    uint32_t seed;
    float clamp_indirect, exposure_scale, inv_spp;
    int view_transform;
    float3 world;
    int n_tris, n_mats;
    // bound on |subpixel offset| of a camera sample (filter support + 1 px of
    // rounding slack): k_tiles' whole-tile culling test
    float filter_reach;
};

// LBVH build for the current obj_xform (uploaded by the caller).
// Stream-ordered; no host synchronisation inside.
// want4: also collapse it into the BVH4 the split path traverses.
// want_ploc: build the PLOC hierarchy instead (large scenes; not with want4).
void build_lbvh(DevScene& s, hipStream_t st, KernelProfiler* prof = nullptr, bool want4 = false,
                bool want_ploc = false);

// Per-frame constants (lights, materials, object transforms; up to
// kUploadMax floats in all) copied into device buffers by one kernel whose
// arguments carry the data (bvh.hip k_upload). A hipMemcpyAsync from pinned
// host memory is a GPU read over PCIe, and such a read queues behind the
// previous frame's 6 MB of device-to-host output writes (PCIe keeps reads
// behind posted writes): measured 112 us per frame on 04vs. Kernel arguments
// are written by the host into device memory, so nothing waits.
constexpr int kUploadMax = 720;
// RR_FLAG_COUNT_TRAVERSAL words: [0..5] traversal totals (nodes, triangles per
// class); k_tiles' counting launch: [6] shader-clock ticks and [7] real-time
// ticks after the scene staging, [8] waves, [9] real-time ticks from entry,
// [10] ~first entry, [11] last end, [12] last entry, [13] ~first end
// (rr_api.cpp fill_stats). (Traversal-stack drops are counted in every
// frame, in the chunk counters: drops_slot.)
constexpr int kTravWords = 14;
// k_tiles' counting launch also logs each box unit u < kUnitLog: words
// kTravWords + 2u / + 2u + 1 = its start / end real-time ticks (rr_debug_tile_costs)
constexpr int kUnitLog = 1 << 16;
struct UploadSeg {
    float* dst;
    int n;
};
bool upload_by_kernarg(const float* src, const UploadSeg* segs, int nseg, hipStream_t st);

// Whether the path kernels take the LDS-resident (fused, BVH2) variant for a
// scene of these sizes; otherwise the split path over the BVH4 in HBM.
bool scene_in_lds(int n_tris, int n_mats, int n_lights);

// Whether render_frame_device renders this frame with k_tiles (one launch over
// all samples; LDS-resident scene). Such a frame touches only per-frame-slot
// buffers and read-only tables, so it may run beside the other slot's frame.
bool frame_uses_tiles(const FrameConsts& base, bool force_wavefront);

// Render all chunks of one frame: film accumulate + tonemap to rgba8.
// counters_per_chunk receives the device counter layout for stats.
void render_frame_device(DevScene& s, DevPaths& p, const FrameConsts& base, int n_chunks,
                         hipStream_t st);

// Trace a batch of rays (debug / parity entry point).
void trace_batch_device(DevScene& s, DevPaths& p, int n, const float4* d_rays, float4* d_hits,
                        int32_t* d_prims, uint8_t* d_occ, hipStream_t st, int width);

// BSDF sampling batch at one shading point (debug / parity entry point).
void bsdf_batch_device(const float* d_mat12, const float* d_lut, const float n3[3], const float wo3[3], int n,
                       const float* d_u, float* d_wi, float* d_f, float* d_pdf, int32_t* d_ok, hipStream_t st);

// sqrt_rn / sqrt_any / rcp_rn (rr_device.h) against sqrtf and 1.0f / x over
// the float bit patterns [lo, lo + n) on the device; d_counts: 5 words
// (rr_debug_fastmath_check).
void fastmath_check_device(uint32_t lo, uint64_t n, unsigned long long* d_counts, hipStream_t st);

// Device JPEG encode (jpeg.hip): the forward transform (tab = dct | qinv luma |
// qinv chroma) + Huffman coding
// of the coefficients into the entropy-coded segment of the file (rows, RSTn
// markers, EOI), written to pinned host memory as [uint64 length][8 B pad]
// [bytes]. d_huff: 4 x 256 packed code | len << 16 (DC luma, AC luma, DC
// chroma, AC chroma; image_io jpeg_huff_tables).
constexpr int kJpegBlockMaxBytes = 216;  // >= the longest coded 8x8 block (1 + 63 x 26 + 27 bits)
struct JpegDevBufs {
    uint32_t* acbits;    // per block: AC bits
    uint32_t* blk_off;   // per block: bit offset in its row
    uint32_t* row_bits;  // mcuy
    uint32_t* ready;     // mcuy: stuffed row length + 1 once counted (k_jpeg_finish)
    uint32_t* scratch;   // mcuy x jpeg_row_scratch_words
};
size_t jpeg_row_scratch_words(int W);
size_t jpeg_stream_max_bytes(int W, int H);
void jpeg_encode_device(const uint8_t* d_rgba, int W, int H, const float* d_tab, const uint32_t* d_huff,
                        int16_t* d_coeffs, JpegDevBufs& b, uint8_t* host_out, hipStream_t st);

// Per chunk: one pair per bounce b = 0..max_bounces {paths entering b+1,
// shadow rays of b}, one pair of slack, then the words below.
int counters_per_chunk(int max_bounces);
// Word of a chunk's counters holding the camera rays traced (counters_per_chunk).
RR_HD int camera_traced_slot(int max_bounces) { return 2 * (max_bounces + 2); }
// Traversal-stack pushes dropped for want of room (every frame; a dropped push
// is a missed subtree, rr_frame_stats.stack_drops).
RR_HD int drops_slot(int max_bounces) { return 2 * (max_bounces + 2) + 1; }
// k_tiles: continuations / shadow rays traversed (two words; the others left
// a hull side of their triangle, hull_flags, and were resolved without one).
RR_HD int escaped_slot(int max_bounces) { return 2 * (max_bounces + 2) + 2; }
int device_cu_count();

}  // namespace rr
