// C ABI of the renderer (include/rr.h). One rr_ctx per GPU; one rr_scene per
// exported project, cached for the worker's lifetime.
//
// Reference behaviour mirrored here (BlenderJobRunner::render_frame,
// /root/reference/worker/src/rendering/runner/mod.rs:72-203 and
// scripts/render-timing-script.py:13-100):
//  * loaded_at            <- time the frame request starts (scene already loaded;
//                            the reference pays a Blender start + .blend read here)
//  * frame_set(N)         -> host animation evaluation (scene.cpp)
//  * started_rendering_at <- before the device work (script :86)
//  * render               -> LBVH build (if transforms changed) + wavefront
//  * finished_rendering_at = file_saving_started_at <- after the 8-bit image is on
//                            the host (utilities.rs:185-192)
//  * write_still          -> JPEG/PNG encode + write, "<path>.jpg|.png"
//  * file_saving_finished_at <- after the write (utilities.rs:195-198)
#include <hip/hip_runtime.h>

#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_set>
#include <vector>

#include "device.hpp"
#include "image_io.hpp"
#include "rr.h"
#include "scene.hpp"
#include "view.hpp"

using namespace rr;

static_assert(kMatLutIntervals == kMatLutN && kMatLutFloatsPerMat == kMatLutStride && kMatLutPsOffset == kMatLutPs,
              "scene.hpp material-table layout must match rr_device.h");

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

double unix_now() {
    using namespace std::chrono;
    return duration_cast<duration<double>>(system_clock::now().time_since_epoch()).count();
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

struct PinnedBuf {
    uint8_t* ptr = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap) return;
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        cap = 0;
        RR_HIP(hipHostMalloc(reinterpret_cast<void**>(&ptr), n, hipHostMallocDefault));
        cap = n;
    }
    ~PinnedBuf() {
        if (ptr) (void)hipHostFree(ptr);
    }
};

}  // namespace

struct FrameRun {
    int W, H, chunks, spp_chunk, tile_slices;
    bool rebuilt;
    float build_ms, trace_ms, readback_ms;
    float render_ms, device_ms;  // ev0 -> ev4 (build + trace + view transform), ev0 -> ev2 (+ device JPEG)
    std::vector<int32_t> counters;
    double kernel_ms[RR_K_CLASSES];
    int32_t kernel_launches[RR_K_CLASSES];
    unsigned long long trav[kTravWords];
};

// One frame between rr_frame_submit and rr_frame_complete: its host-side
// outputs (pinned, so the device-to-host copies stay asynchronous), events,
// kernel profiler and the request. Several slots = the next queued frames render
// while the host encodes and writes the previous one.
struct FrameSlot {
    bool busy = false;
    uint64_t ticket = 0;
    // 0 start, 1 built, 4 image done (before the device JPEG coder), 2 stream
    // work done, 3 outputs on the host (after their copies)
    hipEvent_t ev[5] = {};
    DevBuf<int32_t> counters;  // this frame's ray counters (swapped into DevPaths while enqueuing)
    // this frame's device outputs (swapped into DevPaths / rr_ctx while enqueuing):
    // their copies to the host run while the next frames' kernels write the other
    // slot's, so no frame waits for its predecessor's device-to-host copies
    DevBuf<float4> film;
    DevBuf<uint8_t> rgba8;
    DevBuf<int16_t> coeffs;
    KernelProfiler prof;
    PinnedBuf host_rgba, host_counters, host_upload;
    PinnedBuf host_jpeg;   // device-coded JPEG stream: [uint64 length][pad][bytes]
    FrameSetup fs;
    bool view_substituted = false;  // the scene's view settings not applied in full (view_warning says what)
    std::string view_warning;
    double submit_at = 0.0;         // UNIX time when the device work was enqueued
    bool anchor = false;            // submitted to an idle context: its device start is submit_at
    rr_scene* scene = nullptr;
    std::string out_path, format;
    int quality = 0;
    bool jpeg = false, want_rgba = false, count = false;
    bool unit_logged = false;  // its k_tiles launch wrote the unit log into trav_counts (rr_debug_tile_costs)
    float* film_out = nullptr;
    FrameRun r{};
    rr_frame_timing tm{};
    double anim_ms = 0.0;
    std::chrono::steady_clock::time_point t_call;
    // Device state private to this slot, swapped in while its frame is enqueued
    // (SlotSwap), so that a k_tiles frame can run on the GPU beside the other
    // slot's frame: the slot's own stream, the small per-frame buffers of
    // DevPaths (lights, materials, material tables) and of the JPEG coder, and
    // — for k_tiles frames only — the per-frame products of its scene's
    // hierarchy build (`alt`: everything in DevScene but the uploaded
    // triangles, for the scene `alt_scene`). Frames of the split path never
    // overlap their predecessor, so they use the scene's own copy: a large
    // scene is held once, not once per slot.
    hipStream_t stream = nullptr;
    bool tiles = false;  // this frame renders with k_tiles (may overlap its neighbours)
    DevBuf<float> lights, materials, tile_slab;
    DevBuf<float> mat_lut;  // material tables of this slot's frames (uploaded when they change)
    std::vector<float> mat_lut_cached;
    DevBuf<uint32_t> tile_ctrs, tile_cost;
    DevBuf<int32_t> tile_order, spill;
    DevBuf<unsigned long long> trav_counts;
    DevBuf<uint32_t> jpeg_blk, jpeg_scratch;
    DevScene alt;
    const rr_scene* alt_scene = nullptr;
    void release_private() {
        lights.release();
        materials.release();
        mat_lut.release();
        mat_lut_cached.clear();
        tile_slab.release();
        tile_ctrs.release();
        tile_cost.release();
        tile_order.release();
        spill.release();
        trav_counts.release();
        jpeg_blk.release();
        jpeg_scratch.release();
        alt.release();
        alt = DevScene{};
        alt_scene = nullptr;
    }
};

struct rr_ctx {
    int device = 0;
    // the compute stream the device code enqueues on: slot 0's stream outside
    // frames (inspection entry points), the frame slot's stream while a frame is
    // enqueued (enqueue_frame SlotSwap)
    hipStream_t stream = nullptr;
    DevPaths paths;
    // device JPEG transform (jpeg.hip): tables for the last quality, coefficients
    DevBuf<float> jpeg_tab;
    int jpeg_tab_quality = -1;
    DevBuf<int16_t> jpeg_coeffs;
    // device entropy coder (jpeg.hip): Huffman tables, per-row scratch, stream
    DevBuf<uint32_t> jpeg_huff;
    DevBuf<uint32_t> jpeg_scratch, jpeg_blk;
    std::vector<float> filter_cache;
    float filter_width_cached = -1.f;
    bool srgb_uploaded = false;
    FrameSlot slots[RR_MAX_FRAMES_IN_FLIGHT];
    uint64_t next_ticket = 1;     // tickets are issued in submission order
    uint64_t next_complete = 1;   // the ticket rr_frame_complete expects next
    FrameSlot* last_enqueued = nullptr;  // the slot of the frame enqueued last (its ev[2]: device work done)
    bool in_slot = false;  // a frame is being enqueued: the slot's private buffers are swapped in
    // UNIX-time estimate of when the compute stream finished the last completed
    // frame (rr_frame_complete): the next frame's device work cannot start before
    double gpu_free_at = 0.0;
    FilmicDev filmic;             // RR_VIEW_FILMIC LUTs (rr_set_ocio_config / RR_OCIO_DIR)
    // rr_last_warning = the context's warning (a broken RR_OCIO_DIR, kept for
    // the context's lifetime) + the last completed frame's
    std::string ctx_warning, frame_warning, warning;
    // Device start times of completed frames (rr_frame_complete): every frame
    // also records its start on start_ring[ticket % kStartRing], which outlives
    // the frame slot's own events by a few frames, so the next frame's start is
    // the previous one's plus the device clock's difference between the two.
    static constexpr int kStartRing = 8;
    hipEvent_t start_ring[kStartRing] = {};
    uint64_t chain_ticket = 0;   // last completed frame whose device start is known (0: none)
    double chain_unix = 0.0;     // its device start, UNIX seconds
    double last_render_end = 0.0;  // finished_rendering_at of the last completed frame
    // scenes bound to this context: rr_destroy releases their device buffers
    // and unbinds them, so a scene freed after its context touches no freed state
    std::unordered_set<rr_scene*> scenes;
};

struct rr_scene {
    rr_ctx* ctx = nullptr;
    SceneDesc desc;
    DevScene dev;
};

namespace {

// Catch-all wrapper: C++ exceptions never cross the C ABI.
template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const HipError& e) {
        return fail(RR_ENODEV, e.what());
    } catch (const std::bad_alloc&) {
        return fail(RR_ENOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return fail(RR_EINVAL, e.what());
    }
}

void set_device(rr_ctx* c) { RR_HIP(hipSetDevice(c->device)); }

// Waits for every compute stream of the context (the home stream and both
// slots'; while a frame is enqueued its slot stream sits in c->stream). Called
// before a table that all frames read (filter, sRGB, material, JPEG, Filmic)
// is rewritten, since a frame of the other slot may still be reading it.
void quiesce(rr_ctx* c) {
    RR_HIP(hipStreamSynchronize(c->stream));
    for (auto& sl : c->slots)
        if (sl.stream) RR_HIP(hipStreamSynchronize(sl.stream));
}

// Exchanges the per-frame products of a scene's hierarchy build (transforms,
// world triangles, build scratch, nodes, packed triangles, cache state) between
// the scene and a slot's private set; the uploaded object-space triangles stay.
void swap_products(DevScene& home, DevScene& alt) {
    std::swap(home, alt);
    std::swap(home.tri_local, alt.tri_local);
    std::swap(home.tri_obj, alt.tri_obj);
    std::swap(home.tri_mat, alt.tri_mat);
    std::swap(home.n_tris, alt.n_tris);
    std::swap(home.n_objs, alt.n_objs);
    std::swap(home.uploaded, alt.uploaded);
}

// One-time upload of the scene's object-space triangles.
void upload_scene(rr_ctx* c, rr_scene* s) {
    set_device(c);
    DevScene& d = s->dev;
    if (d.uploaded) return;
    if (d.n_tris > 0) {
        d.tri_local.ensure((size_t)3 * d.n_tris);
        d.tri_obj.ensure((size_t)d.n_tris);
        d.tri_mat.ensure((size_t)d.n_tris);
        RR_HIP(hipMemcpy(d.tri_local.ptr, s->desc.tri_local.data(), s->desc.tri_local.size() * sizeof(float),
                         hipMemcpyHostToDevice));
        RR_HIP(hipMemcpy(d.tri_obj.ptr, s->desc.tri_obj.data(), d.n_tris * sizeof(int32_t), hipMemcpyHostToDevice));
        RR_HIP(hipMemcpy(d.tri_mat.ptr, s->desc.tri_mat.data(), d.n_tris * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    d.uploaded = true;
}

// A scene is used with exactly one context; a host-only handle binds on first use.
void bind_scene(rr_ctx* c, rr_scene* s) {
    if (s->ctx && s->ctx != c) throw std::runtime_error("scene belongs to another context");
    s->ctx = c;
    c->scenes.insert(s);
    upload_scene(c, s);
}

// Upload per-frame constants and (re)build the LBVH if object transforms changed.
// `staging` (pinned, per frame slot) keeps the host-to-device copies
// asynchronous, so a frame can be enqueued while the previous one still runs.
// Hierarchy ids (render_ints[7] of rr_debug_frame_state, rr_debug_trace):
// 2 = Karras LBVH (BVH2), 3 = PLOC (BVH2), 4 = PLOC (LBVH below 3 triangles)
// collapsed to the quantised 6-wide hierarchy (rr_device.h QNode6).
constexpr int kHierLbvh = 2, kHierPloc = 3, kHierQWide = 4;  // 4: the quantised 6-wide collapse (ABI value kept)

FrameConsts make_consts(const FrameSetup& fs, int n_tris);

// The hierarchy the frame kernels walk: the LBVH for frames k_tiles renders
// (LDS-resident scenes), the quantised BVH4 for the split path (larger scenes,
// and LDS-resident ones under RR_FLAG_WAVEFRONT).
int frame_hier(const FrameSetup& fs, int n_tris) {
    return frame_uses_tiles(make_consts(fs, n_tris), (fs.flags & RR_FLAG_WAVEFRONT) != 0) ? kHierLbvh : kHierQWide;
}

// The view transform a frame on ctx is rendered with: Filmic needs the
// context's LUTs, without them Standard. Returns what of the scene's view
// settings the frame does not apply ("" if nothing): that fallback, and the
// scene's own notes (FrameSetup::view_note: an unsupported view transform,
// look or display gamma).
std::string resolve_view(const rr_ctx* c, FrameSetup& fs) {
    std::string w = fs.view_note;
    if (fs.view_transform == VIEW_FILMIC && !(c && c->filmic.ready)) {
        fs.view_transform = VIEW_STANDARD;
        w = "scene view transform Filmic rendered as Standard: no OCIO LUTs configured "
            "(rr_set_ocio_config / RR_OCIO_DIR)" + (w.empty() ? "" : "; " + w);
    }
    return w;
}

// hier: 0 = the frame's hierarchy, else a kHier* id (inspection entry points).
bool prepare_frame(rr_ctx* c, rr_scene* s, const FrameSetup& fs, PinnedBuf& staging, int hier = 0) {
    bind_scene(c, s);
    hipStream_t st = c->stream;
    DevPaths& p = c->paths;
    // tables (built on the host once; identical construction in the oracle)
    if (c->filter_width_cached != fs.filter_width) {
        quiesce(c);
        c->filter_cache.assign(kFilterTableSize, 0.f);
        build_filter_table(fs.filter_width, c->filter_cache.data());
        p.filter_table.ensure(kFilterTableSize);
        RR_HIP(hipMemcpy(p.filter_table.ptr, c->filter_cache.data(), kFilterTableSize * sizeof(float),
                         hipMemcpyHostToDevice));
        c->filter_width_cached = fs.filter_width;
    }
    if (!c->srgb_uploaded) {
        quiesce(c);
        std::vector<float> lut(kSrgbLutSize + 1);
        build_srgb_lut(lut.data());
        p.srgb_lut.ensure(lut.size());
        RR_HIP(hipMemcpy(p.srgb_lut.ptr, lut.data(), lut.size() * sizeof(float), hipMemcpyHostToDevice));
        c->srgb_uploaded = true;
    }
    if (p.mat_lut_cached != fs.mat_lut) {  // material tables: static per scene, uploaded when they change
        // a frame slot's own table is read only by that slot's frames (the
        // slot's previous frame has completed); the context's table, used by
        // the inspection calls, may be read by any stream
        if (!c->in_slot) quiesce(c);
        p.mat_lut.ensure(fs.mat_lut.size());
        RR_HIP(hipMemcpyAsync(p.mat_lut.ptr, fs.mat_lut.data(), fs.mat_lut.size() * sizeof(float),
                              hipMemcpyHostToDevice, st));
        RR_HIP(hipStreamSynchronize(st));  // pageable source: the copy must be done before fs goes away
        p.mat_lut_cached = fs.mat_lut;
    }
    const size_t nl = fs.lights.size(), nm = fs.materials.size(), nx = fs.obj_xform.size();
    p.lights.ensure(nl ? nl : 1);
    p.materials.ensure(nm ? nm : 1);
    staging.ensure((nl + nm + nx) * sizeof(float));
    float* up = reinterpret_cast<float*>(staging.ptr);
    std::memcpy(up, fs.lights.data(), nl * sizeof(float));
    std::memcpy(up + nl, fs.materials.data(), nm * sizeof(float));
    std::memcpy(up + nl + nm, fs.obj_xform.data(), nx * sizeof(float));
    DevScene& d = s->dev;
    if (hier == 0) hier = frame_hier(fs, d.n_tris);
    const bool want4 = hier == kHierQWide;
    const bool want_ploc = (hier == kHierPloc || hier == kHierQWide) && d.n_tris > 2;
    // (a BVH4 collapse reorders the triangles into its leaf order, so a BVH2
    // walk of the same PLOC tree needs a build without it)
    const bool rebuild = !d.built || d.cached_xform != fs.obj_xform || (want4 != d.has4) || (want_ploc != d.ploc);
    const bool upload_x = rebuild && d.n_tris > 0;
    if (upload_x) d.obj_xform.ensure(nx);
    const UploadSeg segs[3] = {{p.lights.ptr, (int)nl}, {p.materials.ptr, (int)nm},
                               {upload_x ? d.obj_xform.ptr : nullptr, upload_x ? (int)nx : 0}};
    if (!upload_by_kernarg(up, segs, 3, st)) {
        if (nl) RR_HIP(hipMemcpyAsync(p.lights.ptr, up, nl * sizeof(float), hipMemcpyHostToDevice, st));
        RR_HIP(hipMemcpyAsync(p.materials.ptr, up + nl, nm * sizeof(float), hipMemcpyHostToDevice, st));
        if (upload_x)
            RR_HIP(hipMemcpyAsync(d.obj_xform.ptr, up + nl + nm, nx * sizeof(float), hipMemcpyHostToDevice, st));
    }
    if (upload_x) {
        build_lbvh(d, st, &p.prof, want4, want_ploc);
        d.cached_xform = fs.obj_xform;
    } else if (rebuild) {
        d.built = true;
        d.cached_xform = fs.obj_xform;
    }
    return rebuild;
}

FrameConsts make_consts(const FrameSetup& fs, int n_tris) {
    FrameConsts k{};
    k.cam_pos = make_float3(fs.cam[0], fs.cam[1], fs.cam[2]);
    k.cam_right = make_float3(fs.cam[3], fs.cam[4], fs.cam[5]);
    k.cam_up = make_float3(fs.cam[6], fs.cam[7], fs.cam[8]);
    k.cam_back = make_float3(fs.cam[9], fs.cam[10], fs.cam[11]);
    k.half_w = fs.cam[12];
    k.half_h = fs.cam[13];
    k.clip_start = fs.cam[14];
    k.clip_end = fs.cam[15];
    k.inv_w2 = 2.0f / (float)fs.W;
    k.inv_h2 = 2.0f / (float)fs.H;
    k.W = fs.W;
    k.H = fs.H;
    k.npix = fs.W * fs.H;
    k.div_w = FastDiv::make((uint32_t)fs.W);
    k.div_spp = FastDiv::make(1u);  // per chunk (render_split)
    k.spp_total = fs.spp;
    k.max_bounces = fs.max_bounces;
    k.max_diffuse = fs.max_diffuse;
    k.max_glossy = fs.max_glossy;
    k.n_lights = (int)(fs.lights.size() / RR_LIGHT_FLOATS);
    k.n_mats = (int)(fs.materials.size() / RR_MAT_FLOATS);
    k.seed = fs.seed;
    k.clamp_indirect = fs.clamp_indirect;
    k.exposure_scale = fs.exposure_scale;
    k.inv_spp = 1.0f / (float)fs.spp;
    k.view_transform = fs.view_transform;
    k.world = make_float3(fs.world[0], fs.world[1], fs.world[2]);
    k.n_tris = n_tris;
    // build_filter_table: offsets within the support [-width, width]
    k.filter_reach = std::fabs(fs.filter_width) + 1.0f;
    return k;
}

int choose_spp_chunk(const FrameSetup& fs) {
    if (fs.spp_per_chunk > 0) return std::min(fs.spp_per_chunk, fs.spp);
    // Paths in flight per chunk: the SoA path state is 168 B/path (radiance
    // record 16 B, two path-queue slots 2 x 48 B, shadow slot 48 B, hit 8 B),
    // so the default 512M paths take ~86 GB of the 288 GB HBM (a 1080p frame
    // up to 256 spp, a 4K frame's 64 spp, is one chunk; frames of the split
    // path share one copy); np stays below 2^31 for 32-bit queue indices.
    // Per full C5 frame (4K, 1024 spp) 256M / 512M / 1G paths per chunk:
    // 4,113 / 4,016 / 4,088 ms (profiles/r5_ab_chunk.txt): half the launches
    // and their tails.
#ifndef RR_CHUNK_MPATHS
#define RR_CHUNK_MPATHS 512
#endif
    constexpr long kChunkPaths = (long)RR_CHUNK_MPATHS << 20;
    const long target = kChunkPaths;
    long c = target / std::max(1, fs.W * fs.H);
    if (c < 1) c = 1;
    if (c > fs.spp) c = fs.spp;
    return (int)c;
}

// The chunk a frame renders with: choose_spp_chunk, lowered when the path
// state of that many paths (168 B each, DevPaths::ensure_paths) would not fit
// in 85 % of the device memory free now plus what this context's path buffers
// already hold — a smaller GPU, or several ranks sharing one, gets more chunks
// instead of RR_ENOMEM. Chunking changes no bit of the image
// (test_chunking_and_determinism); an explicit spp_per_chunk is kept as asked.
int fit_spp_chunk(const FrameSetup& fs, const DevPaths& p) {
    const int c = choose_spp_chunk(fs);
    if (fs.spp_per_chunk > 0) return c;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return c;
    }
    constexpr size_t kPathStateBytes = 168;
    const double usable = 0.85 * ((double)free_b + (double)p.cap * kPathStateBytes);
    const double npix = std::max(1.0, (double)fs.W * fs.H);
    // ensure_paths' slack: a persistent grid's threads + 1/64 of the paths
    const double slack = (double)std::max(p.grid_blocks, 256 * 8) * kBlock;  // 8: kMaxBlocksPerCu
    const long fit = (long)((usable / kPathStateBytes - slack) / (1.0 + 1.0 / 64.0) / npix);
    return (int)std::max<long>(1, std::min<long>(c, fit));
}

// Device JPEG encode of an RGBA8 frame (transform into c->jpeg_coeffs +
// Huffman coding) into the slot's pinned stream buffer, on the context stream.
void enqueue_jpeg_device(rr_ctx* c, FrameSlot& sl, const uint8_t* d_rgba, int W, int H, const float* d_tab) {
    if (!c->jpeg_huff.ptr) {
        quiesce(c);
        uint32_t h[4 * 256];
        jpeg_huff_tables(h);
        c->jpeg_huff.ensure(4 * 256);
        RR_HIP(hipMemcpy(c->jpeg_huff.ptr, h, sizeof h, hipMemcpyHostToDevice));
    }
    const size_t mcuy = (size_t)(H + 15) / 16;
    const size_t nblocks = mcuy * (size_t)((W + 15) / 16) * 6;
    c->jpeg_coeffs.ensure(jpeg_coeff_count(W, H));
    c->jpeg_blk.ensure(2 * nblocks + 2 * mcuy);
    c->jpeg_scratch.ensure(mcuy * jpeg_row_scratch_words(W));
    sl.host_jpeg.ensure(jpeg_stream_max_bytes(W, H) + 16);
    void* dev_host = nullptr;
    RR_HIP(hipHostGetDevicePointer(&dev_host, sl.host_jpeg.ptr, 0));
    uint32_t* blk = c->jpeg_blk.ptr;
    JpegDevBufs b{blk, blk + nblocks, blk + 2 * nblocks, blk + 2 * nblocks + mcuy, c->jpeg_scratch.ptr};
    jpeg_encode_device(d_rgba, W, H, d_tab, c->jpeg_huff.ptr, c->jpeg_coeffs.ptr, b, static_cast<uint8_t*>(dev_host),
                       c->stream);
}

// The file of a device-coded frame: host-built header + the device stream.
bool write_device_jpeg(const FrameSlot& sl, const std::string& path, uint64_t* bytes) {
    uint64_t len = 0;
    std::memcpy(&len, sl.host_jpeg.ptr, sizeof len);
    if (len + 16 > sl.host_jpeg.cap) throw std::runtime_error("device JPEG stream overflow");
    std::vector<uint8_t> data;
    jpeg_header_bytes(sl.fs.W, sl.fs.H, sl.quality, data);
    data.insert(data.end(), sl.host_jpeg.ptr + 16, sl.host_jpeg.ptr + 16 + len);
    *bytes = data.size();
    return write_file(path, data);
}

// Enqueue the device part of one frame on the context stream (no host
// synchronisation): LBVH (if needed), wavefront, tonemap, optionally the JPEG
// transform, and the asynchronous copies of the slot's outputs.
void enqueue_frame(rr_ctx* c, FrameSlot& sl) {
    set_device(c);
    rr_scene* s = sl.scene;
    const FrameSetup& fs = sl.fs;
    FrameRun& r = sl.r;
    r = FrameRun{};
    r.W = fs.W;
    r.H = fs.H;
    for (auto& e : sl.ev)
        if (!e) RR_HIP(hipEventCreate(&e));
    if (sl.alt_scene != s) {  // products of another scene (or none): start this scene's set afresh
        sl.alt.release();
        sl.alt = DevScene{};
        sl.alt_scene = s;
    }
    // This frame runs on its slot's stream with the slot's private buffers
    // swapped in (the other slot's frame may still be running). A k_tiles frame
    // following a k_tiles frame does not wait for it: k_tiles and its helper
    // kernels touch only slot buffers and read-only tables, so frame N+1's
    // build and launch fill the CUs that frame N's tail and its JPEG kernels
    // leave idle. Any other frame shares the wavefront queues of DevPaths and
    // waits for the previous frame's device work.
    struct SlotSwap {
        rr_ctx* c;
        FrameSlot& sl;
        void swap() {
            DevPaths& p = c->paths;
            std::swap(c->stream, sl.stream);
            std::swap(p.lights, sl.lights);
            std::swap(p.materials, sl.materials);
            std::swap(p.mat_lut, sl.mat_lut);
            std::swap(p.mat_lut_cached, sl.mat_lut_cached);
            std::swap(p.tile_slab, sl.tile_slab);
            std::swap(p.tile_ctrs, sl.tile_ctrs);
            std::swap(p.tile_cost, sl.tile_cost);
            std::swap(p.tile_order, sl.tile_order);
            std::swap(p.spill, sl.spill);
            std::swap(p.trav_counts, sl.trav_counts);
            std::swap(c->jpeg_blk, sl.jpeg_blk);
            std::swap(c->jpeg_scratch, sl.jpeg_scratch);
            if (sl.tiles) swap_products(sl.scene->dev, sl.alt);
            c->in_slot = !c->in_slot;
        }
        SlotSwap(rr_ctx* c_, FrameSlot& s_) : c(c_), sl(s_) { swap(); }
        ~SlotSwap() { swap(); }
    };
    sl.tiles = frame_uses_tiles(make_consts(fs, s->dev.n_tris), (fs.flags & RR_FLAG_WAVEFRONT) != 0);
    SlotSwap slot_swap(c, sl);
    hipStream_t st = c->stream;
    FrameSlot* prev = c->last_enqueued;
    if (prev && prev != &sl && !(sl.tiles && prev->tiles))
        RR_HIP(hipStreamWaitEvent(st, prev->ev[2], 0));
    c->last_enqueued = &sl;
    // a k_tiles frame enqueued while another k_tiles frame is pending overlaps
    // it: whole-tile work units (render_frame_device); a frame rendered alone
    // (rr_render_frame, the first of a batch) slices its tiles by sample group.
    // Scheduling only: both give the same bits.
    bool pending_tiles = false;
    for (auto& o : c->slots)
        if (&o != &sl && o.busy && o.tiles) pending_tiles = true;
    c->paths.tile_whole = sl.tiles && pending_tiles;
    sl.prof.reset((fs.flags & RR_FLAG_PROFILE_KERNELS) != 0);
    struct ProfSwap {  // the device code records into paths.prof; swapped back on every exit
        KernelProfiler &a, &b;
        ProfSwap(KernelProfiler& x, KernelProfiler& y) : a(x), b(y) { std::swap(a, b); }
        ~ProfSwap() { std::swap(a, b); }
    } prof_swap(c->paths.prof, sl.prof);
    struct CtrSwap {  // per-slot counters: the previous frame's may still be on their way to the host
        DevBuf<int32_t>&a, &b;
        CtrSwap(DevBuf<int32_t>& x, DevBuf<int32_t>& y) : a(x), b(y) { std::swap(a, b); }
        ~CtrSwap() { std::swap(a, b); }
    } ctr_swap(c->paths.counters, sl.counters);
    struct OutSwap {  // per-slot output buffers (film, rgba8, JPEG coefficients)
        rr_ctx* c;
        FrameSlot& sl;
        void swap() {
            std::swap(c->paths.film, sl.film);
            std::swap(c->paths.rgba8, sl.rgba8);
            std::swap(c->jpeg_coeffs, sl.coeffs);
        }
        OutSwap(rr_ctx* c_, FrameSlot& s_) : c(c_), sl(s_) { swap(); }
        ~OutSwap() { swap(); }
    } out_swap(c, sl);
    sl.count = (fs.flags & RR_FLAG_COUNT_TRAVERSAL) != 0;
    c->paths.count_traversal = sl.count;
    c->paths.force_wavefront = (fs.flags & RR_FLAG_WAVEFRONT) != 0;
    RR_HIP(hipEventRecord(sl.ev[0], st));
    {
        hipEvent_t& se = c->start_ring[sl.ticket % rr_ctx::kStartRing];
        if (!se) RR_HIP(hipEventCreate(&se));
        RR_HIP(hipEventRecord(se, st));
    }
    r.rebuilt = prepare_frame(c, s, fs, sl.host_upload);
    RR_HIP(hipEventRecord(sl.ev[1], st));
    FrameConsts k = make_consts(fs, s->dev.n_tris);
    r.spp_chunk = fit_spp_chunk(fs, c->paths);
    r.chunks = (fs.spp + r.spp_chunk - 1) / r.spp_chunk;
    k.spp_chunk = r.spp_chunk;
    k.div_spp = FastDiv::make((uint32_t)k.spp_chunk);
    render_frame_device(s->dev, c->paths, k, r.chunks, st);
    r.tile_slices = c->paths.last_tile_slices;
    sl.unit_logged = c->paths.last_unit_logged;
    if (fs.view_transform == VIEW_FILMIC) {  // film -> Filmic -> rgba8 (overwrites the kernels' tonemap)
        c->paths.prof.begin(st, RR_K_ACCUM);
        view_filmic_device(c->filmic, k, c->paths.film.ptr, reinterpret_cast<uchar4*>(c->paths.rgba8.ptr), st);
        c->paths.prof.end(st);
    }
    RR_HIP(hipEventRecord(sl.ev[4], st));
    const size_t npix = (size_t)fs.W * fs.H;
    if (sl.jpeg) {
        if (c->jpeg_tab_quality != sl.quality) {
            quiesce(c);
            JpegTables t;
            jpeg_tables(sl.quality, t);
            float tab[192];
            std::memcpy(tab, t.dct, sizeof t.dct);
            std::memcpy(tab + 64, t.qinv_l, sizeof t.qinv_l);
            std::memcpy(tab + 128, t.qinv_c, sizeof t.qinv_c);
            c->jpeg_tab.ensure(192);
            RR_HIP(hipMemcpy(c->jpeg_tab.ptr, tab, sizeof tab, hipMemcpyHostToDevice));
            c->jpeg_tab_quality = sl.quality;
        }
        enqueue_jpeg_device(c, sl, c->paths.rgba8.ptr, fs.W, fs.H, c->jpeg_tab.ptr);
    }
    RR_HIP(hipEventRecord(sl.ev[2], st));
    // the outputs' device-to-host copies follow on the slot's own stream: the
    // next frames run on the other slots' streams, so nothing waits for them
    hipStream_t cs = st;
    if (sl.want_rgba) {
        sl.host_rgba.ensure(npix * 4);
        RR_HIP(hipMemcpyAsync(sl.host_rgba.ptr, c->paths.rgba8.ptr, npix * 4, hipMemcpyDeviceToHost, cs));
    }
    const int cpc = counters_per_chunk(fs.max_bounces);
    const size_t nctr = (size_t)cpc * r.chunks;
    sl.host_counters.ensure(nctr * sizeof(int32_t));
    RR_HIP(hipMemcpyAsync(sl.host_counters.ptr, c->paths.counters.ptr, nctr * sizeof(int32_t), hipMemcpyDeviceToHost,
                          cs));
    if (sl.film_out)
        RR_HIP(hipMemcpyAsync(sl.film_out, c->paths.film.ptr, npix * sizeof(float4), hipMemcpyDeviceToHost, cs));
    RR_HIP(hipEventRecord(sl.ev[3], cs));
    if (sl.count) {  // measurement mode: read the traversal counters now
        RR_HIP(hipStreamSynchronize(st));
        RR_HIP(hipMemcpy(r.trav, c->paths.trav_counts.ptr, sizeof r.trav, hipMemcpyDeviceToHost));
        c->paths.count_traversal = false;
    }
}

// Wait for a slot's device work and collect its timings and counters.
void finish_frame(rr_ctx* c, FrameSlot& sl) {
    set_device(c);
    FrameRun& r = sl.r;
    const FrameSetup& fs = sl.fs;
    RR_HIP(hipEventSynchronize(sl.ev[3]));
    RR_HIP(hipEventElapsedTime(&r.build_ms, sl.ev[0], sl.ev[1]));
    RR_HIP(hipEventElapsedTime(&r.trace_ms, sl.ev[1], sl.ev[4]));
    RR_HIP(hipEventElapsedTime(&r.readback_ms, sl.ev[4], sl.ev[3]));
    RR_HIP(hipEventElapsedTime(&r.render_ms, sl.ev[0], sl.ev[4]));
    RR_HIP(hipEventElapsedTime(&r.device_ms, sl.ev[0], sl.ev[2]));
    const int cpc = counters_per_chunk(fs.max_bounces);
    r.counters.assign(reinterpret_cast<const int32_t*>(sl.host_counters.ptr),
                      reinterpret_cast<const int32_t*>(sl.host_counters.ptr) + (size_t)cpc * r.chunks);
    sl.prof.collect(r.kernel_ms, r.kernel_launches);
    sl.prof.reset(false);
    if (sl.film_out) {  // film holds sums; report the mean
        const size_t npix = (size_t)fs.W * fs.H;
        const float inv = 1.0f / (float)fs.spp;
        for (size_t i = 0; i < npix; ++i) {
            float* f = sl.film_out + 4 * i;
            f[0] = f[0] * inv;
            f[1] = f[1] * inv;
            f[2] = f[2] * inv;
            f[3] = 1.0f;
        }
    }
}

void fill_stats(rr_frame_stats* st, const FrameSetup& fs, const FrameRun& r, int n_tris) {
    if (!st) return;
    std::memset(st, 0, sizeof *st);
    st->width = fs.W;
    st->height = fs.H;
    st->spp = fs.spp;
    st->chunks = r.chunks;
    st->camera_rays = (uint64_t)fs.W * fs.H * fs.spp;
    st->view_transform = fs.view_transform;
    const int cpc = counters_per_chunk(fs.max_bounces);
    uint64_t drops = 0, ext_traced = 0, sh_traced = 0;
    for (int c = 0; c < r.chunks; ++c) {
        // pair b: {paths entering bounce b+1, shadow rays of bounce b} (wavefront.hip)
        const int32_t* q = &r.counters[(size_t)cpc * c];
        st->camera_rays_traced += (uint64_t)(uint32_t)q[camera_traced_slot(fs.max_bounces)];
        drops += (uint64_t)(uint32_t)q[drops_slot(fs.max_bounces)];
        if (r.tile_slices > 0) {  // k_tiles: the traversed ones are counted; the rest escaped
            ext_traced += (uint64_t)(uint32_t)q[escaped_slot(fs.max_bounces)];
            sh_traced += (uint64_t)(uint32_t)q[escaped_slot(fs.max_bounces) + 1];
        }
        for (int b = 0; b < fs.max_bounces; ++b) st->extension_rays += (uint64_t)q[2 * b];
        for (int b = 0; b <= fs.max_bounces; ++b) st->shadow_rays += (uint64_t)q[2 * b + 1];
        st->primary_continued += (uint64_t)q[0];
        st->primary_shadow += (uint64_t)q[1];
    }
    for (int k = 0; k < RR_K_CLASSES; ++k) {
        st->kernel_ms[k] = r.kernel_ms[k];
        st->kernel_launches[k] = r.kernel_launches[k];
    }
    for (int k = 0; k < 3; ++k) {
        st->trav_nodes[k] = r.trav[2 * k];
        st->trav_tris[k] = r.trav[2 * k + 1];
    }
    {
        // k_tiles<count>: sums over waves of shader-clock and 100 MHz real-time ticks
        const unsigned long long* w = r.trav;
        st->kernel_clock_ghz = w[7] ? 0.1 * (double)w[6] / (double)w[7] : 0.0;
        const unsigned long long t0 = ~w[10], t1 = w[11];
        st->kernel_wave_fill = (w[8] && t1 > t0) ? (double)w[9] / (double)w[8] / (double)(t1 - t0) : 0.0;
        const unsigned long long e1 = w[12], x0 = ~w[13];
        st->kernel_entry_spread = (w[8] && t1 > t0 && e1 >= t0) ? (double)(e1 - t0) / (double)(t1 - t0) : 0.0;
        st->kernel_exit_spread = (w[8] && t1 > t0 && t1 >= x0) ? (double)(t1 - x0) / (double)(t1 - t0) : 0.0;
    }
    st->stack_drops = (int32_t)std::min<uint64_t>(drops, 0x7fffffffull);
    if (r.tile_slices > 0) {
        st->extension_rays_escaped = st->extension_rays - std::min(ext_traced, st->extension_rays);
        st->shadow_rays_escaped = st->shadow_rays - std::min(sh_traced, st->shadow_rays);
    }
    st->build_ms = r.rebuilt ? r.build_ms : 0.0;
    st->trace_ms = r.trace_ms;
    st->readback_ms = r.readback_ms;
    st->bvh_rebuilt = r.rebuilt ? 1 : 0;
    st->tile_slices = r.tile_slices;
    st->n_triangles = n_tris;
}

int do_encode(const uint8_t* rgba, int W, int H, const char* out_path, const char* format, int quality,
              uint64_t* bytes) {
    if (!out_path || !format) return fail(RR_EINVAL, "out_path and format are required");
    const std::string fmt(format);
    std::vector<uint8_t> data;
    std::string ext;
    if (fmt == "JPEG") {
        if (quality < 1 || quality > 100) return fail(RR_EINVAL, "jpeg_quality must be 1..100");
        if (!encode_jpeg(rgba, W, H, quality, data)) return fail(RR_EINVAL, "JPEG encode failed");
        ext = ".jpg";
    } else if (fmt == "PNG") {
        if (!encode_png(rgba, W, H, data, 1)) return fail(RR_EIO, "PNG encode failed");
        ext = ".png";
    } else {
        return fail(RR_ENOTSUP, "unsupported output format '" + fmt + "' (JPEG and PNG are supported)");
    }
    const std::string path = std::string(out_path) + ext;
    if (!write_file(path, data)) return fail(RR_EIO, "cannot write " + path + ": " + std::strerror(errno));
    if (bytes) *bytes = data.size();
    return RR_OK;
}

// BVH width the frame kernels traverse for this scene (2: LDS-resident fused
// path, 4: split path from HBM).
int frame_hier_of(rr_scene* s, const FrameSetup& fs) { return frame_hier(fs, s->dev.n_tris); }

FrameSlot* slot_for(rr_ctx* c, uint64_t ticket) { return &c->slots[ticket % RR_MAX_FRAMES_IN_FLIGHT]; }

bool idle(rr_ctx* c) { return c->next_complete == c->next_ticket; }

}  // namespace

extern "C" {

void rr_render_params_default(rr_render_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->spp = 0;
    p->max_bounces = -1;
    p->clamp_indirect = -1.0f;
    p->seed = 0;
    p->use_scene_seed = 1;
    p->width = 0;
    p->height = 0;
    p->view_transform = RR_VIEW_SCENE;
    p->spp_per_chunk = 0;
    p->max_diffuse_bounces = -1;
    p->max_glossy_bounces = -1;
}

int32_t rr_abi_version(void) { return RR_ABI_VERSION; }

const char* rr_last_error(rr_ctx*) { return g_err.c_str(); }

const char* rr_last_warning(rr_ctx* c) {
    if (!c) return "";
    c->warning = c->ctx_warning;
    if (!c->frame_warning.empty()) c->warning += (c->warning.empty() ? "" : "; ") + c->frame_warning;
    return c->warning.c_str();
}

int rr_set_ocio_config(rr_ctx* c, const char* dir) {
    if (!c) return fail(RR_EINVAL, "NULL ctx");
    return guarded([&] {
        set_device(c);
        quiesce(c);
        c->filmic.release();
        c->ctx_warning.clear();  // an RR_OCIO_DIR problem is superseded by this call
        if (!dir || !*dir) return RR_OK;
        FilmicLuts l;
        std::string err;
        if (!load_filmic_luts(dir, l, err)) return fail(err.rfind("no ", 0) == 0 || err.rfind("cannot", 0) == 0 ? RR_ENOENT : RR_EINVAL, err);
        c->filmic.upload(l, dir);
        return RR_OK;
    });
}

int rr_create(int device_ordinal, rr_ctx** out) {
    if (!out) return fail(RR_EINVAL, "out is NULL");
    *out = nullptr;
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RR_ENODEV, "no HIP device available");
        if (device_ordinal < 0 || device_ordinal >= n)
            return fail(RR_ENODEV, "device ordinal " + std::to_string(device_ordinal) + " out of range (" +
                                       std::to_string(n) + " visible)");
        std::unique_ptr<rr_ctx> c(new rr_ctx());
        c->device = device_ordinal;
        set_device(c.get());
        // One stream per slot and no other, so that each gets a hardware queue
        // of its own (GPU_MAX_HW_QUEUES is 4, and the process's null stream
        // holds one): streams created beyond that share a queue, and a queue
        // runs its kernels in order, so frames of two slots on one queue
        // cannot overlap. The home stream (inspection calls) is slot 0's;
        // with RR_MAX_FRAMES_IN_FLIGHT = 3 the three slots and the null stream
        // take the four queues.
        for (auto& sl : c->slots) RR_HIP(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
        c->stream = c->slots[0].stream;
        if (const char* d = getenv("RR_OCIO_DIR")) {
            // a broken LUT directory does not fail the context: Filmic frames fall
            // back to Standard and carry the reason in rr_last_warning
            FilmicLuts l;
            std::string err;
            if (*d && load_filmic_luts(d, l, err)) c->filmic.upload(l, d);
            else if (*d) c->ctx_warning = "RR_OCIO_DIR: " + err;
        }
        *out = c.release();
        return RR_OK;
    });
}

void rr_destroy(rr_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& sl : c->slots)
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
    c->paths.release();
    c->filmic.release();
    c->jpeg_tab.release();
    c->jpeg_coeffs.release();
    c->jpeg_huff.release();
    c->jpeg_scratch.release();
    c->jpeg_blk.release();
    for (auto& sl : c->slots) {
        for (auto& e : sl.ev)
            if (e) (void)hipEventDestroy(e);
        sl.prof.release();
    }
    for (auto& e : c->start_ring)
        if (e) (void)hipEventDestroy(e);
    for (rr_scene* s : c->scenes) {  // still-open scenes: back to host-only handles
        s->dev.release();
        s->ctx = nullptr;
    }
    for (auto& sl : c->slots) {
        if (sl.stream) (void)hipStreamDestroy(sl.stream);  // c->stream is slot 0's
        sl.release_private();
        sl.counters.release();
        sl.film.release();
        sl.rgba8.release();
        sl.coeffs.release();
    }
    delete c;
}

int rr_scene_load(rr_ctx* c, const char* path, rr_scene** out) {
    if (!path || !out) return fail(RR_EINVAL, "NULL argument");
    *out = nullptr;
    {
        FILE* f = std::fopen(path, "rb");
        if (!f) return fail(RR_ENOENT, std::string("scene file doesn't exist: ") + path);
        std::fclose(f);
    }
    return guarded([&] {
        std::unique_ptr<rr_scene> s(new rr_scene());
        s->desc = load_scene(path);
        s->dev.n_tris = (int)s->desc.tri_obj.size();
        s->dev.n_objs = (int)s->desc.objects.size();
        if (c) bind_scene(c, s.get());  // NULL: host-only handle, bound to a context at its first render
        *out = s.release();
        return RR_OK;
    });
}

void rr_scene_free(rr_scene* s) {
    if (!s) return;
    if (rr_ctx* c = s->ctx) {
        (void)hipSetDevice(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        for (auto& sl : c->slots) {
            if (sl.stream) (void)hipStreamSynchronize(sl.stream);
            if (sl.alt_scene == s) {  // the slot's build products of this scene
                sl.alt.release();
                sl.alt = DevScene{};
                sl.alt_scene = nullptr;
            }
        }
        c->scenes.erase(s);
    }
    s->dev.release();
    delete s;
}

int rr_scene_resolution(rr_scene* s, const rr_render_params* p, int32_t* w, int32_t* h) {
    if (!s) return fail(RR_EINVAL, "scene is NULL");
    return guarded([&] {
        rr_render_params d;
        rr_render_params_default(&d);
        const RenderDesc& r = s->desc.render;
        const int W = (p && p->width > 0) ? p->width : (r.resx * r.percent) / 100;
        const int H = (p && p->height > 0) ? p->height : (r.resy * r.percent) / 100;
        if (w) *w = W;
        if (h) *h = H;
        return RR_OK;
    });
}

int rr_frame_submit(rr_ctx* c, rr_scene* s, int32_t frame, const rr_render_params* params, const char* out_path,
                    const char* format, int32_t jpeg_quality, uint64_t* ticket) {
    if (!c || !s || !ticket) return fail(RR_EINVAL, "NULL ctx, scene or ticket");
    if (s->ctx && s->ctx != c) return fail(RR_EINVAL, "scene belongs to another context");
    if (out_path && !format) return fail(RR_EINVAL, "format is required when out_path is given");
    if (format && std::string(format) != "JPEG" && std::string(format) != "PNG")
        return fail(RR_ENOTSUP, std::string("unsupported output format '") + format + "'");
    const bool jpeg = out_path && std::string(format) == "JPEG";
    if (jpeg && (jpeg_quality < 1 || jpeg_quality > 100)) return fail(RR_EINVAL, "jpeg_quality must be 1..100");
    FrameSlot* sl = slot_for(c, c->next_ticket);
    if (sl->busy) return fail(RR_EBUSY, "too many frames in flight (complete the oldest first)");
    return guarded([&] {
        sl->t_call = std::chrono::steady_clock::now();
        sl->tm = rr_frame_timing{};
        sl->tm.loaded_at = unix_now();
        const auto t_anim = std::chrono::steady_clock::now();
        sl->fs = setup_frame(s->desc, frame, params);
        sl->view_warning = resolve_view(c, sl->fs);
        sl->view_substituted = !sl->view_warning.empty();
        sl->anim_ms = ms_since(t_anim);
        sl->tm.started_rendering_at = unix_now();
        sl->scene = s;
        sl->out_path = out_path ? out_path : "";
        sl->format = (out_path && format) ? format : "";
        sl->quality = jpeg_quality;
        sl->jpeg = jpeg;
        sl->want_rgba = out_path && !jpeg;
        sl->film_out = nullptr;
        sl->anchor = idle(c);
        sl->submit_at = unix_now();
        sl->ticket = c->next_ticket;
        enqueue_frame(c, *sl);
        sl->busy = true;
        ++c->next_ticket;
        *ticket = sl->ticket;
        return RR_OK;
    });
}

int rr_frame_complete(rr_ctx* c, uint64_t ticket, rr_frame_timing* timing, rr_frame_stats* stats) {
    if (!c) return fail(RR_EINVAL, "NULL ctx");
    if (ticket != c->next_complete) return fail(RR_EINVAL, "frames must be completed in submission order");
    FrameSlot* sl = slot_for(c, ticket);
    if (!sl->busy || sl->ticket != ticket) return fail(RR_EINVAL, "unknown ticket");
    auto release = [&] {
        sl->busy = false;
        c->next_complete = ticket + 1;
    };
    const int rc = guarded([&] {
        finish_frame(c, *sl);
        const FrameSetup& fs = sl->fs;
        const FrameRun& r = sl->r;
        const double t_sync = unix_now();
        // Render span from the device's own clock. The frame's device work
        // starts at its start event: for a frame submitted to an idle context
        // that is the submit time; otherwise the previous completed frame's
        // device start plus the device clock's difference between the two
        // start events (start_ring). Frames in flight together overlap on the
        // device, but the worker's records are consecutive (traces.py
        // not_before, performance.rs): the render span starts when the
        // previous frame's ended, or at the device start if later, and ends
        // at the frame's own end event (ev4: build, trace, view transform),
        // so the spans of overlapped frames add up to at most the wall time
        // they took. The device JPEG coder, the copies and the file write
        // after ev4 are "saving" (Blender's write_still).
        constexpr int K = rr_ctx::kStartRing;
        double dev_start = std::max(sl->submit_at, c->gpu_free_at);
        if (!sl->anchor && c->chain_ticket && c->chain_ticket + 1 == ticket && c->start_ring[ticket % K]) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, c->start_ring[c->chain_ticket % K], c->start_ring[ticket % K]) == hipSuccess)
                dev_start = c->chain_unix + ms * 1e-3;
        }
        dev_start = std::min(std::max(dev_start, sl->submit_at), t_sync);
        c->chain_ticket = ticket;
        c->chain_unix = dev_start;
        sl->tm.started_rendering_at = std::min(std::max(dev_start, c->last_render_end), t_sync);
        sl->tm.finished_rendering_at =
            std::min(std::max(dev_start + r.render_ms * 1e-3, sl->tm.started_rendering_at), t_sync);
        sl->tm.file_saving_started_at = sl->tm.finished_rendering_at;
        c->last_render_end = sl->tm.finished_rendering_at;
        c->gpu_free_at = std::min(dev_start + r.device_ms * 1e-3, t_sync);
        uint64_t bytes = 0;
        const auto t_enc = std::chrono::steady_clock::now();
        if (sl->jpeg) {  // JFIF headers + the device-coded stream
            const std::string path = sl->out_path + ".jpg";
            if (!write_device_jpeg(*sl, path, &bytes))
                return fail(RR_EIO, "cannot write " + path + ": " + std::strerror(errno));
        } else if (!sl->out_path.empty()) {
            const int e = do_encode(sl->host_rgba.ptr, fs.W, fs.H, sl->out_path.c_str(), sl->format.c_str(),
                                    sl->quality, &bytes);
            if (e != RR_OK) return e;
        }
        const double enc_ms = ms_since(t_enc);
        sl->tm.file_saving_finished_at = unix_now();
        if (timing) *timing = sl->tm;
        c->frame_warning = sl->view_warning;
        if (stats) {
            fill_stats(stats, fs, r, sl->scene->dev.n_tris);
            stats->view_transform_substituted = sl->view_substituted ? 1 : 0;
            stats->anim_ms = sl->anim_ms;
            stats->encode_ms = enc_ms;
            stats->output_bytes = bytes;
            stats->total_ms = ms_since(sl->t_call);
        }
        return RR_OK;
    });
    release();
    return rc;
}

int rr_render_frame(rr_ctx* c, rr_scene* s, int32_t frame, const rr_render_params* params, const char* out_path,
                    const char* format, int32_t jpeg_quality, rr_frame_timing* timing, rr_frame_stats* stats) {
    if (c && c->next_complete != c->next_ticket)
        return fail(RR_EBUSY, "rr_render_frame while submitted frames are pending");
    uint64_t t = 0;
    const int rc = rr_frame_submit(c, s, frame, params, out_path, format, jpeg_quality, &t);
    if (rc != RR_OK) return rc;
    return rr_frame_complete(c, t, timing, stats);
}

int rr_synchronize(rr_ctx* c) {
    if (!c) return fail(RR_EINVAL, "NULL ctx");
    return guarded([&] {
        set_device(c);
        quiesce(c);
        return RR_OK;
    });
}

int rr_render_frame_to_memory(rr_ctx* c, rr_scene* s, int32_t frame, const rr_render_params* params,
                              float* film, uint8_t* rgba8, rr_frame_stats* stats) {
    if (!c || !s) return fail(RR_EINVAL, "NULL ctx or scene");
    if (s->ctx && s->ctx != c) return fail(RR_EINVAL, "scene belongs to another context");
    if (c->next_complete != c->next_ticket) return fail(RR_EBUSY, "submitted frames are pending");
    FrameSlot* sl = slot_for(c, c->next_ticket);
    return guarded([&] {
        sl->t_call = std::chrono::steady_clock::now();
        sl->fs = setup_frame(s->desc, frame, params);
        sl->view_warning = resolve_view(c, sl->fs);
        sl->view_substituted = !sl->view_warning.empty();
        sl->scene = s;
        sl->out_path.clear();
        sl->format.clear();
        sl->jpeg = false;
        sl->want_rgba = true;
        sl->film_out = film;
        sl->ticket = c->next_ticket;
        enqueue_frame(c, *sl);
        finish_frame(c, *sl);
        sl->film_out = nullptr;
        const FrameSetup& fs = sl->fs;
        if (rgba8) std::memcpy(rgba8, sl->host_rgba.ptr, (size_t)fs.W * fs.H * 4);
        c->frame_warning = sl->view_warning;
        if (stats) {
            fill_stats(stats, fs, sl->r, s->dev.n_tris);
            stats->view_transform_substituted = sl->view_substituted ? 1 : 0;
            stats->total_ms = ms_since(sl->t_call);
        }
        return RR_OK;
    });
}

int rr_encode_image(const uint8_t* rgba8, int32_t w, int32_t h, const char* out_path, const char* format,
                    int32_t quality, uint64_t* bytes) {
    if (!rgba8 || w <= 0 || h <= 0) return fail(RR_EINVAL, "bad image");
    return guarded([&] { return do_encode(rgba8, w, h, out_path, format, quality, bytes); });
}

int rr_debug_jpeg_device(rr_ctx* c, const uint8_t* rgba8, int32_t w, int32_t h, int32_t quality, uint8_t* out,
                         uint64_t cap, uint64_t* len) {
    if (!c || !rgba8 || !len || w <= 0 || h <= 0 || w > 65535 || h > 65535) return fail(RR_EINVAL, "bad arguments");
    if (quality < 1 || quality > 100) return fail(RR_EINVAL, "jpeg_quality must be 1..100");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        set_device(c);
        hipStream_t st = c->stream;
        DevBuf<uint8_t> img;
        img.ensure((size_t)w * h * 4);
        RR_HIP(hipMemcpy(img.ptr, rgba8, (size_t)w * h * 4, hipMemcpyHostToDevice));
        JpegTables t;
        jpeg_tables(quality, t);
        float tab[192];
        std::memcpy(tab, t.dct, sizeof t.dct);
        std::memcpy(tab + 64, t.qinv_l, sizeof t.qinv_l);
        std::memcpy(tab + 128, t.qinv_c, sizeof t.qinv_c);
        DevBuf<float> dtab;
        dtab.ensure(192);
        RR_HIP(hipMemcpy(dtab.ptr, tab, sizeof tab, hipMemcpyHostToDevice));
        c->jpeg_tab_quality = -1;  // the context's cached table is not this one's
        FrameSlot& sl = c->slots[0];
        sl.fs.W = w;
        sl.fs.H = h;
        sl.quality = quality;
        enqueue_jpeg_device(c, sl, img.ptr, w, h, dtab.ptr);
        RR_HIP(hipStreamSynchronize(st));
        uint64_t n = 0;
        std::memcpy(&n, sl.host_jpeg.ptr, sizeof n);
        std::vector<uint8_t> hdr;
        jpeg_header_bytes(w, h, quality, hdr);
        *len = hdr.size() + n;
        if (out && cap >= *len) {
            std::memcpy(out, hdr.data(), hdr.size());
            std::memcpy(out + hdr.size(), sl.host_jpeg.ptr + 16, n);
        }
        img.release();
        dtab.release();
        return RR_OK;
    });
}

int rr_debug_scene_mesh(rr_scene* s, float* tri_local9, int32_t* tri_object) {
    if (!s) return fail(RR_EINVAL, "scene is NULL");
    const size_t n = s->desc.tri_obj.size();
    if (tri_local9)
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k)
                for (int a = 0; a < 3; ++a) tri_local9[9 * i + 3 * k + a] = s->desc.tri_local[12 * i + 4 * k + a];
    if (tri_object && n) std::memcpy(tri_object, s->desc.tri_obj.data(), n * sizeof(int32_t));
    return RR_OK;
}

int rr_debug_counts(rr_scene* s, int32_t* nt, int32_t* nl, int32_t* nm, int32_t* no) {
    if (!s) return fail(RR_EINVAL, "scene is NULL");
    int lights = 0;
    for (auto& o : s->desc.objects) lights += o.type == OBJ_LIGHT;
    if (nt) *nt = (int32_t)s->desc.tri_obj.size();
    if (nl) *nl = lights;
    if (nm) *nm = (int32_t)s->desc.materials.size();
    if (no) *no = (int32_t)s->desc.objects.size();
    return RR_OK;
}

int rr_debug_frame_state(rr_ctx* c, rr_scene* s, int32_t frame, const rr_render_params* params, float* tris_world,
                         int32_t* tri_material, float* camera, float* lights, float* materials, float* world,
                         int32_t* render_ints, float* render_floats) {
    if (!s) return fail(RR_EINVAL, "NULL scene");
    if (!c && tris_world) return fail(RR_EINVAL, "world triangles need a device context");
    return guarded([&] {
        FrameSetup fs = setup_frame(s->desc, frame, params);
        if (c) resolve_view(c, fs);  // render_ints[5]: the transform a frame on c is rendered with
        const int n = s->dev.n_tris;
        if (c) {  // host-only queries (c == NULL) skip the device part
            if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
            set_device(c);
            PinnedBuf staging;
            prepare_frame(c, s, fs, staging);
            RR_HIP(hipStreamSynchronize(c->stream));
        }
        if (tris_world && n > 0) {
            std::vector<float4> w((size_t)3 * n);
            RR_HIP(hipMemcpyAsync(w.data(), s->dev.tri_world.ptr, w.size() * sizeof(float4), hipMemcpyDeviceToHost,
                                  c->stream));
            RR_HIP(hipStreamSynchronize(c->stream));
            for (size_t i = 0; i < w.size(); ++i) {
                tris_world[3 * i] = w[i].x;
                tris_world[3 * i + 1] = w[i].y;
                tris_world[3 * i + 2] = w[i].z;
            }
        }
        if (c) RR_HIP(hipStreamSynchronize(c->stream));
        if (tri_material) std::memcpy(tri_material, s->desc.tri_mat.data(), n * sizeof(int32_t));
        if (camera) std::memcpy(camera, fs.cam, sizeof fs.cam);
        if (lights && !fs.lights.empty()) std::memcpy(lights, fs.lights.data(), fs.lights.size() * sizeof(float));
        if (materials) std::memcpy(materials, fs.materials.data(), fs.materials.size() * sizeof(float));
        if (world) std::memcpy(world, fs.world, sizeof fs.world);
        if (render_ints) {
            const int32_t ri[RR_RENDER_INTS] = {fs.W, fs.H, fs.spp, fs.max_bounces, (int32_t)fs.seed,
                                               fs.view_transform, choose_spp_chunk(fs), frame_hier_of(s, fs),
                                               fs.max_diffuse, fs.max_glossy};
            std::memcpy(render_ints, ri, sizeof ri);
        }
        if (render_floats) {
            const float rf[RR_RENDER_FLOATS] = {fs.clamp_indirect, fs.filter_width, fs.exposure_scale, 0.f};
            std::memcpy(render_floats, rf, sizeof rf);
        }
        return RR_OK;
    });
}

int rr_debug_bvh(rr_ctx* c, rr_scene* s, int32_t frame, uint32_t* keys, uint32_t* order, int32_t* children,
                 float* boxes) {
    return rr_debug_bvh_hier(c, s, frame, 0, keys, order, children, boxes);
}

int rr_debug_bvh_hier(rr_ctx* c, rr_scene* s, int32_t frame, int32_t hier, uint32_t* keys, uint32_t* order,
                      int32_t* children, float* boxes) {
    if (!c || !s) return fail(RR_EINVAL, "NULL ctx or scene");
    if (hier != 0 && hier != kHierLbvh && hier != kHierPloc) return fail(RR_EINVAL, "hier must be 0, 2 or 3");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        FrameSetup fs = setup_frame(s->desc, frame, nullptr);
        set_device(c);
        PinnedBuf staging;
        prepare_frame(c, s, fs, staging, hier);
        DevScene& d = s->dev;
        const int n = d.n_tris;
        hipStream_t st = c->stream;
        if (n > 0) {
            if (keys) RR_HIP(hipMemcpyAsync(keys, d.keys[0].ptr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            if (order) RR_HIP(hipMemcpyAsync(order, d.vals[0].ptr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            const int ni = n > 1 ? n - 1 : 1;
            std::vector<BvhNode> nodes((size_t)ni);
            RR_HIP(hipMemcpyAsync(nodes.data(), d.nodes.ptr, ni * sizeof(BvhNode), hipMemcpyDeviceToHost, st));
            RR_HIP(hipStreamSynchronize(st));
            for (int i = 0; i < ni; ++i) {
                const float* f = reinterpret_cast<const float*>(&nodes[i]);
                if (boxes) std::memcpy(boxes + 12 * i, f, 12 * sizeof(float));
                if (children) {
                    children[2 * i] = nodes[i].d.x;
                    children[2 * i + 1] = nodes[i].d.y;
                }
            }
        }
        RR_HIP(hipStreamSynchronize(st));
        return RR_OK;
    });
}

int rr_debug_qbvh(rr_ctx* c, rr_scene* s, int32_t frame, int32_t* nq, int32_t* children, uint32_t* nodes16,
                  int32_t* tri_orig) {
    if (!c || !s || !nq) return fail(RR_EINVAL, "NULL ctx, scene or nq");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        FrameSetup fs = setup_frame(s->desc, frame, nullptr);
        set_device(c);
        PinnedBuf staging;
        prepare_frame(c, s, fs, staging, kHierQWide);
        DevScene& d = s->dev;
        hipStream_t st = c->stream;
        const int n = d.n_tris;
        *nq = 0;
        if (n > 0) {
            const uint32_t cnt = (uint32_t)d.nq;
            *nq = (int32_t)cnt;
            if (children || nodes16) {
                std::vector<QNode6> nodes(cnt);
                RR_HIP(hipMemcpyAsync(nodes.data(), d.qnodes.ptr, cnt * sizeof(QNode6), hipMemcpyDeviceToHost, st));
                RR_HIP(hipStreamSynchronize(st));
                for (uint32_t i = 0; i < cnt; ++i) {
                    const QNode6& q = nodes[i];
                    if (children) {  // the implicit references, spelled out (unused slots: 0x7fffffff)
                        const uint32_t eb = (uint32_t)f2i(q.org.w);
                        for (int k = 0; k < kQWidth; ++k) {
                            const uint32_t lox = k < 4 ? (q.a.z >> (8 * k)) & 255u : (q.c.x >> (8 * (k - 4))) & 255u;
                            const uint32_t hix = k < 4 ? (q.b.y >> (8 * k)) & 255u : (q.c.y >> (16 + 8 * (k - 4))) & 255u;
                            const bool unused = lox == 255u && hix == 0u && !((eb >> (24 + k)) & 1u);
                            children[kQWidth * (size_t)i + k] = unused ? 0x7fffffff : q6_ref(q, k);
                        }
                    }
                    if (nodes16) std::memcpy(nodes16 + 16 * (size_t)i, &q, sizeof(QNode6));
                }
            }
            if (tri_orig) {  // original id of each position of the hierarchy's triangle array
                std::vector<TriPack> tp((size_t)n);
                RR_HIP(hipMemcpyAsync(tp.data(), d.tris.ptr, (size_t)n * sizeof(TriPack), hipMemcpyDeviceToHost, st));
                RR_HIP(hipStreamSynchronize(st));
                for (int i = 0; i < n; ++i) tri_orig[i] = f2i(tp[(size_t)i].p0.w);
            }
        }
        return RR_OK;
    });
}

int rr_debug_trace(rr_ctx* c, rr_scene* s, int32_t frame, int32_t bvh_width, int32_t n, const float* rays,
                   float* hits, int32_t* prims, uint8_t* occluded) {
    if (!c || !s || n < 0 || (n > 0 && !rays)) return fail(RR_EINVAL, "bad arguments");
    if (bvh_width < 0 || bvh_width == 1 || bvh_width > 7)
        return fail(RR_EINVAL, "hierarchy must be 0 (frame's), 2 (LBVH), 3 (PLOC), 4 (6-wide), 5 (6-wide, packets) "
                               "6 (6-wide, one LDS stack entry) or 7 (6-wide, beam packets)");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        FrameSetup fs = setup_frame(s->desc, frame, nullptr);
        set_device(c);
        PinnedBuf staging;
        const int hier = bvh_width >= 5 ? kHierQWide : (bvh_width ? bvh_width : frame_hier_of(s, fs));
        prepare_frame(c, s, fs, staging, hier);
        const int width = bvh_width >= 5 ? bvh_width : (hier == kHierQWide ? 4 : 2);
        hipStream_t st = c->stream;
        DevBuf<float4> dr, dh;
        DevBuf<int32_t> dp;
        DevBuf<uint8_t> dq;
        const size_t m = n > 0 ? (size_t)n : 1;
        dr.ensure(2 * m);
        dh.ensure(m);
        dp.ensure(m);
        dq.ensure(m);
        if (n > 0) RR_HIP(hipMemcpyAsync(dr.ptr, rays, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice, st));
        trace_batch_device(s->dev, c->paths, n, dr.ptr, dh.ptr, dp.ptr, dq.ptr, st, width);
        std::vector<float4> h(m);
        if (n > 0) {
            RR_HIP(hipMemcpyAsync(h.data(), dh.ptr, n * sizeof(float4), hipMemcpyDeviceToHost, st));
            if (prims) RR_HIP(hipMemcpyAsync(prims, dp.ptr, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
            if (occluded) RR_HIP(hipMemcpyAsync(occluded, dq.ptr, n, hipMemcpyDeviceToHost, st));
        }
        RR_HIP(hipStreamSynchronize(st));
        if (hits)
            for (int i = 0; i < n; ++i) {
                hits[4 * i] = h[i].x;
                hits[4 * i + 1] = h[i].y;
                hits[4 * i + 2] = h[i].z;
                hits[4 * i + 3] = 0.0f;
            }
        dr.release(); dh.release(); dp.release(); dq.release();
        return RR_OK;
    });
}

int rr_debug_tile_costs(rr_ctx* c, int32_t capacity, uint32_t* costs, int32_t* order, int32_t* n_tiles,
                        uint64_t* unit_log, int32_t unit_capacity) {
    if (!c || capacity < 0 || !n_tiles || (capacity > 0 && (!costs || !order)) || unit_capacity < 0 ||
        (unit_capacity > 0 && !unit_log))
        return fail(RR_EINVAL, "bad arguments");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        *n_tiles = 0;
        const FrameSlot* sl = c->last_enqueued;
        if (!sl || !sl->tiles) return RR_OK;  // no tile frame yet
        set_device(c);
        const size_t n = std::min(sl->tile_cost.cap, sl->tile_order.cap);
        *n_tiles = (int32_t)n;
        const size_t m = std::min<size_t>(n, (size_t)capacity);
        if (m > 0) {
            RR_HIP(hipMemcpy(costs, sl->tile_cost.ptr, m * sizeof(uint32_t), hipMemcpyDeviceToHost));
            RR_HIP(hipMemcpy(order, sl->tile_order.ptr, m * sizeof(int32_t), hipMemcpyDeviceToHost));
        }
        const size_t nu = std::min<size_t>((size_t)unit_capacity, kUnitLog);
        if (nu > 0) {
            std::memset(unit_log, 0, 2 * nu * sizeof(uint64_t));
            // only the launch that wrote it (a counting frame): an older frame's log stays unreported
            if (sl->unit_logged && sl->trav_counts.cap >= (size_t)(kTravWords + 2 * kUnitLog))
                RR_HIP(hipMemcpy(unit_log, sl->trav_counts.ptr + kTravWords, 2 * nu * sizeof(uint64_t),
                                 hipMemcpyDeviceToHost));
        }
        return RR_OK;
    });
}

int rr_debug_fastmath_check(rr_ctx* c, uint32_t lo, uint64_t n, uint64_t* counts5) {
    if (!c || !counts5 || n > (1ull << 32) - lo) return fail(RR_EINVAL, "bad arguments");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        set_device(c);
        hipStream_t st = c->stream;
        DevBuf<unsigned long long> d;
        d.ensure(5);
        fastmath_check_device(lo, n, d.ptr, st);
        RR_HIP(hipMemcpyAsync(counts5, d.ptr, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        RR_HIP(hipStreamSynchronize(st));
        d.release();
        return RR_OK;
    });
}

int rr_debug_bsdf_sample(rr_ctx* c, const float* mat12, const float* n3, const float* wo3, int32_t n,
                         const float* u, float* wi3, float* f3, float* pdf, int32_t* ok) {
    if (!c || !mat12 || !n3 || !wo3 || n < 0 || (n > 0 && (!u || !wi3 || !f3 || !pdf || !ok)))
        return fail(RR_EINVAL, "bad arguments");
    return guarded([&] {
        if (!idle(c)) return fail(RR_EBUSY, "submitted frames are pending");
        set_device(c);
        hipStream_t st = c->stream;
        const size_t m = n > 0 ? (size_t)n : 1;
        DevBuf<float> dm, du, dw, df, dp, dl;
        DevBuf<int32_t> dk;
        float lut[kMatLutFloatsPerMat];
        build_material_lut(mat12, lut);
        dl.ensure(kMatLutFloatsPerMat);
        RR_HIP(hipMemcpyAsync(dl.ptr, lut, sizeof lut, hipMemcpyHostToDevice, st));
        dm.ensure(RR_MAT_FLOATS);
        du.ensure(3 * m); dw.ensure(3 * m); df.ensure(3 * m); dp.ensure(m); dk.ensure(m);
        RR_HIP(hipMemcpyAsync(dm.ptr, mat12, RR_MAT_FLOATS * sizeof(float), hipMemcpyHostToDevice, st));
        if (n > 0) RR_HIP(hipMemcpyAsync(du.ptr, u, 3 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, st));
        bsdf_batch_device(dm.ptr, dl.ptr, n3, wo3, n, du.ptr, dw.ptr, df.ptr, dp.ptr, dk.ptr, st);
        if (n > 0) {
            RR_HIP(hipMemcpyAsync(wi3, dw.ptr, 3 * (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
            RR_HIP(hipMemcpyAsync(f3, df.ptr, 3 * (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
            RR_HIP(hipMemcpyAsync(pdf, dp.ptr, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
            RR_HIP(hipMemcpyAsync(ok, dk.ptr, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        }
        RR_HIP(hipStreamSynchronize(st));
        RR_HIP(hipStreamSynchronize(st));
        dm.release(); du.release(); dw.release(); df.release(); dp.release(); dk.release(); dl.release();
        return RR_OK;
    });
}

int rr_debug_object_matrix(rr_scene* s, int32_t obj, double frame, double* m16) {
    if (!s || !m16) return fail(RR_EINVAL, "NULL argument");
    return guarded([&] {
        object_matrix(s->desc, obj, frame, m16);
        return RR_OK;
    });
}

}  // extern "C"
