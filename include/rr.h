/*
 * rr.h — C ABI of the MI355X frame renderer ("rr" = render-runner backend).
 *
 * This is the drop-in boundary for the one hot path of the render cluster: the
 * worker's per-frame render step. In the reference that step is a process
 * boundary: BlenderJobRunner::render_frame spawns `blender <blend> --background
 * --python render-timing-script.py -- --render-output … --render-format …
 * --render-frame N` and parses its stdout
 * (/root/reference/worker/src/rendering/runner/mod.rs:72-203, argv :140-158,
 * spawn :165-174; stdout protocol worker/src/rendering/runner/utilities.rs:105-203).
 * Here the same step is an in-process call: scene exported once per project,
 * uploaded once, then rr_render_frame() per frame index.
 *
 * Plain C types only (no torch / HIP types). All functions return 0 on success
 * and a negative errno-style code on failure; rr_last_error() then holds a
 * UTF-8 message (thread-local, valid until the next call on this thread).
 *
 * Threading: one rr_ctx per GPU per process; a ctx is NOT thread-safe, calls on
 * one ctx must be serialised by the caller (the reference worker renders one
 * frame at a time per worker: worker/src/rendering/queue.rs:79-118).
 * Ownership: the caller owns ctx and scene handles (Rust Drop -> rr_scene_free /
 * rr_destroy).
 */
#ifndef RR_H
#define RR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RR_ABI_VERSION 8

/* error codes (negative errno values) */
#define RR_OK 0
#define RR_ENOENT (-2)   /* file missing (reference: runner/mod.rs:82-87, :99-104) */
#define RR_EIO (-5)      /* read/write failure (reference: create_dir_all :117-121) */
#define RR_ENOMEM (-12)  /* host or device allocation failure */
#define RR_EINVAL (-22)  /* bad argument / malformed scene */
#define RR_ENODEV (-19)  /* HIP device unavailable / kernel launch failure */
#define RR_ENOTSUP (-95) /* unsupported output format or scene feature */
#define RR_EBUSY (-16)   /* rr_frame_submit with RR_MAX_FRAMES_IN_FLIGHT frames pending */

/* Frames a context keeps between rr_frame_submit and rr_frame_complete. */
#define RR_MAX_FRAMES_IN_FLIGHT 3

typedef struct rr_ctx rr_ctx;
typedef struct rr_scene rr_scene;

/* View transform selector (scene "view_transform"). */
#define RR_VIEW_SCENE (-1)  /* use the scene file's setting */
#define RR_VIEW_STANDARD 0  /* sRGB OETF, Blender "Standard" */
#define RR_VIEW_RAW 1       /* linear values, clamped, no OETF */
#define RR_VIEW_FILMIC 2    /* Blender "Filmic" (display sRGB, look None) through the OCIO LUTs of a
                             * Blender colour-management directory (rr_set_ocio_config); without
                             * them the frame is rendered with Standard and flagged
                             * (rr_frame_stats.view_transform_substituted, rr_last_warning) */

/* Render parameters. Any field left at its "use scene" value takes the value
 * exported from the project (scene file "render" block). Zero-initialising the
 * struct and then calling rr_render_params_default() gives scene defaults. */
typedef struct rr_render_params {
    int32_t spp;            /* samples per pixel; <= 0: scene */
    int32_t max_bounces;    /* path length cap; < 0: scene */
    float clamp_indirect;   /* max component of indirect contributions; < 0: scene; 0: off */
    uint32_t seed;          /* RNG seed (Cycles "seed") */
    int32_t use_scene_seed; /* != 0: ignore .seed, use the scene's */
    int32_t width;          /* <= 0: scene resolution_x * percentage */
    int32_t height;         /* <= 0: scene resolution_y * percentage */
    int32_t view_transform; /* RR_VIEW_* */
    int32_t spp_per_chunk;  /* samples in flight per wavefront chunk; <= 0: auto */
    int32_t flags;          /* RR_FLAG_* (measurement modes; 0 in production) */
    int32_t max_diffuse_bounces; /* Cycles max_diffuse_bounces (scene default 4); < 0: scene */
    int32_t max_glossy_bounces;  /* Cycles max_glossy_bounces (scene default 4); < 0: scene */
} rr_render_params;

/* Measurement flags (rr_render_params.flags). */
#define RR_FLAG_PROFILE_KERNELS 1  /* HIP events around every launch -> stats.kernel_ms[] */
#define RR_FLAG_COUNT_TRAVERSAL 2  /* count BVH nodes visited / triangles tested -> stats */
#define RR_FLAG_WAVEFRONT 4        /* LDS-resident scenes: the split trace/shade kernels of large scenes
                                    * (quantised BVH4 from HBM) instead of k_tiles (parity: both paths) */

/* Kernel classes of rr_frame_stats.kernel_ms / kernel_launches. */
#define RR_K_BUILD 0     /* world transform + Morton + radix sort + Karras + refit */
#define RR_K_PRIMARY 1   /* bounce 0: raygen + closest hit + shade + queue compaction */
#define RR_K_EXTEND 2    /* bounces >= 1: closest hit + shade + queue compaction */
#define RR_K_SHADOW 3    /* any-hit traversal of shadow rays */
#define RR_K_ACCUM 4     /* film accumulate + tonemap */
#define RR_K_SHADE 5     /* split path (large scenes): shading kernels; PRIMARY/EXTEND then time traversal only */
#define RR_K_TILES 6     /* LDS-resident scenes: k_tiles, every sample of an 8x8 pixel tile run to completion + film + tonemap */
#define RR_K_CLASSES 8

/* The five timestamps the reference recovers from Blender's stdout
 * (PartialRenderStatistics, worker/src/rendering/runner/utilities.rs:14-20,
 * derived at :177-194). UNIX seconds as f64, the serde representation of
 * FrameRenderTime (shared/src/results/worker_trace.rs:13-34). The caller adds
 * started_process_at / exited_process_at around the call exactly as
 * runner/mod.rs:165,176 do. */
typedef struct rr_frame_timing {
    double loaded_at;              /* reference: script start, render-timing-script.py:13 */
    double started_rendering_at;   /* reference: :86 */
    double finished_rendering_at;  /* reference: project_finished_rendering_at - saving (utilities.rs:185-190) */
    double file_saving_started_at; /* == finished_rendering_at (utilities.rs:191-192) */
    double file_saving_finished_at;/* reference: project_finished_rendering_at (utilities.rs:195-198) */
} rr_frame_timing;

/* Per-frame statistics (sidecar metrics; never part of the trace JSON). */
typedef struct rr_frame_stats {
    int32_t width, height, spp, chunks;
    uint64_t camera_rays;    /* camera samples, W * H * spp (camera_rays_traced: those traversed) */
    uint64_t extension_rays; /* continuation rays spawned (closest hit); extension_rays_escaped of them
                              * are resolved without a traversal */
    uint64_t shadow_rays;    /* NEE shadow rays spawned (any hit); shadow_rays_escaped of them are
                              * resolved without a traversal */
    uint64_t primary_continued; /* camera paths that continue past bounce 0 */
    uint64_t primary_shadow;    /* shadow rays spawned at bounce 0 */
    double anim_ms;          /* host animation eval + upload */
    double build_ms;         /* device: world transform + LBVH build (0 if cached) */
    double trace_ms;         /* device: wavefront kernels (raygen .. accumulate) */
    double readback_ms;      /* device->host of the 8-bit image */
    double encode_ms;        /* host: JPEG/PNG encode + write */
    double total_ms;         /* whole call */
    int32_t bvh_rebuilt;     /* 1 if the LBVH was rebuilt for this frame */
    int32_t n_triangles;
    uint64_t output_bytes;   /* encoded file size */
    /* RR_FLAG_PROFILE_KERNELS: summed device time and launch count per class */
    double kernel_ms[RR_K_CLASSES];
    int32_t kernel_launches[RR_K_CLASSES];
    /* RR_FLAG_COUNT_TRAVERSAL: BVH nodes visited / triangles tested over the
     * frame, per traversal kernel: [0] primary, [1] extend, [2] shadow */
    uint64_t trav_nodes[3], trav_tris[3];
    /* camera rays actually traced: camera_rays counts W*H*spp, of which the
     * ones outside the scene's screen rectangle (or meeting no triangle of
     * their tile) are resolved as background without a traversal */
    uint64_t camera_rays_traced;
    int32_t view_transform;            /* RR_VIEW_* the frame was rendered with */
    int32_t view_transform_substituted;/* 1: the scene asked for Filmic, no LUTs were configured, Standard used */
    /* RR_FLAG_COUNT_TRAVERSAL, LDS-resident scenes: the shader clock the tile
     * kernel ran at, in GHz, measured inside it (shader-clock ticks over the
     * 100 MHz real-time counter across each wave's lifetime, summed over waves);
     * 0 when not measured */
    double kernel_clock_ghz;
    /* same launch: the waves' mean lifetime over the launch's span (first wave
     * start to last wave end), i.e. how full the persistent grid stayed; 0
     * when not measured */
    double kernel_wave_fill;
    /* LDS-resident scenes (k_tiles): work units per tile of the scene's
     * screen box — 1 when the frame overlapped another k_tiles frame in flight
     * (whole tiles, every sample group of a tile in one unit), the number of
     * 32-sample groups when it ran alone (one unit per group); 0 for frames of
     * the other paths. Scheduling only: both give the same bits. */
    int32_t tile_slices;
    /* traversal-stack pushes dropped for want of room over the frame (each a
     * missed subtree; counted in every frame; 0 on every bench scene) */
    int32_t stack_drops;
    /* LDS-resident scenes (k_tiles): continuation / shadow rays of extension_rays /
     * shadow_rays that leave a hull side of their triangle (every vertex of the
     * scene lies behind that side's plane), so they meet nothing and are
     * resolved without a traversal (the continuation adds the world term, the
     * shadow ray is unoccluded). Rays that entered a traversal =
     * camera_rays_traced + extension_rays - extension_rays_escaped + shadow_rays
     * - shadow_rays_escaped. 0 on the split path (every ray is traversed). */
    uint64_t extension_rays_escaped;
    uint64_t shadow_rays_escaped;
    /* RR_FLAG_COUNT_TRAVERSAL, LDS-resident scenes (with kernel_wave_fill):
     * the spread of the tile kernel's wave starts (last start - first start)
     * and of its wave ends (last end - first end), each over the launch's span;
     * 0 when not measured */
    double kernel_entry_spread;
    double kernel_exit_spread;
} rr_frame_stats;

/* Fill p with "use the scene's value" for every field. */
void rr_render_params_default(rr_render_params* p);

/* Library / ABI version (RR_ABI_VERSION). */
int32_t rr_abi_version(void);

/* Create a renderer context on HIP device `device_ordinal` (index among the
 * devices visible to this process). */
int rr_create(int device_ordinal, rr_ctx** out);

/* Load a scene exported once per project (".rrscene" JSON)
 * and upload its meshes to ctx's device. ctx may be NULL: the handle is then
 * host-only (animation / resolution queries) and binds to the first context
 * that renders it. The reference re-reads the .blend on
 * every frame (runner/mod.rs:142-146); here the scene is parsed and uploaded
 * once and cached in the returned handle. */
int rr_scene_load(rr_ctx* ctx, const char* scene_path, rr_scene** out);

/* Render one frame. Replaces the Blender subprocess of runner/mod.rs:140-174
 * plus scene.frame_set / render(write_still=True) of render-timing-script.py:81-92.
 *  - frame_index: the frame to evaluate (Blender frame number, scene.frame_set).
 *  - out_path: output path WITHOUT extension, '#' runs already substituted
 *    (render-timing-script.py:69-78,82); the library appends ".jpg" / ".png"
 *    as Blender's write_still does with R_EXTENSION. NULL: render only.
 *  - format: "JPEG" or "PNG" (job output_file_format, shared/src/jobs/mod.rs:80).
 *  - jpeg_quality: 1..100 (the reference script forces 90, :84).
 *  - timing / stats: optional outputs (may be NULL). */
int rr_render_frame(rr_ctx* ctx, rr_scene* scene, int32_t frame_index,
                    const rr_render_params* params, const char* out_path,
                    const char* format, int32_t jpeg_quality,
                    rr_frame_timing* timing, rr_frame_stats* stats);

/* Two-phase form of rr_render_frame, for a worker that keeps its next queued
 * frame in flight (eager-naive-coarse and dynamic keep
 * frames queued per worker, master/src/cluster/strategies.rs:70-150,250-405,
 * while the reference worker renders them strictly one after another,
 * worker/src/rendering/queue.rs:79-118). rr_frame_submit evaluates the
 * animation, enqueues the frame's device work and returns without waiting;
 * rr_frame_complete waits for that frame's device work, encodes and writes
 * the image and fills timing/stats exactly as rr_render_frame does. The
 * intended loop is submit(N+1), complete(N): the host encodes and writes
 * frame N while the GPU renders N+1. At most RR_MAX_FRAMES_IN_FLIGHT frames
 * may be pending (RR_EBUSY otherwise); they complete in submission order.
 * Each pending frame has its own stream: with three pending, frame N+2's
 * device work is queued while N+1 renders, and starts on the CUs N+1 leaves
 * idle before N's JPEG kernels (waiting behind N+1) have let the host
 * complete N.
 * rr_render_frame == submit + complete. Same arguments and errors as
 * rr_render_frame; a failed complete still retires its ticket. */
int rr_frame_submit(rr_ctx* ctx, rr_scene* scene, int32_t frame_index,
                    const rr_render_params* params, const char* out_path,
                    const char* format, int32_t jpeg_quality, uint64_t* ticket);
int rr_frame_complete(rr_ctx* ctx, uint64_t ticket, rr_frame_timing* timing,
                      rr_frame_stats* stats);

/* Wait until every piece of device work ctx has enqueued (frames in flight
 * included) has finished; their tickets still have to be completed. */
int rr_synchronize(rr_ctx* ctx);

/* Render one frame into caller memory (no file). film_rgba: W*H*4 floats of
 * mean linear radiance (alpha = 1); rgba8: W*H*4 bytes after the view
 * transform. Either may be NULL. Rows are top to bottom. */
int rr_render_frame_to_memory(rr_ctx* ctx, rr_scene* scene, int32_t frame_index,
                              const rr_render_params* params, float* film_rgba,
                              uint8_t* rgba8, rr_frame_stats* stats);

/* Resolved output size for these params (after scene defaults). */
int rr_scene_resolution(rr_scene* scene, const rr_render_params* params,
                        int32_t* width, int32_t* height);

/* Encode an RGBA8 image (rows top to bottom) to `path` + extension.
 * Host encoder used by rr_render_frame; exported for tests. */
int rr_encode_image(const uint8_t* rgba8, int32_t width, int32_t height,
                    const char* out_path_no_ext, const char* format,
                    int32_t jpeg_quality, uint64_t* bytes_written);

/* Encode an RGBA8 image with the device JPEG path (forward DCT + Huffman
 * coding on the GPU, jpeg.hip; the path rr_render_frame takes for "JPEG").
 * *len receives the file size; the bytes are copied to out if cap >= *len.
 * Exported for parity tests against rr_encode_image. */
int rr_debug_jpeg_device(rr_ctx* ctx, const uint8_t* rgba8, int32_t width, int32_t height,
                         int32_t jpeg_quality, uint8_t* out, uint64_t cap, uint64_t* len);

/* Thread-local message of the last failure on this thread (ctx may be NULL). */
const char* rr_last_error(rr_ctx* ctx);

/* Warning of ctx's last completed frame ("" if none), e.g. a Filmic view
 * transform rendered as Standard because no OCIO LUTs are configured. Valid
 * until the next call on ctx. */
const char* rr_last_warning(rr_ctx* ctx);

/* Blender colour-management directory (datafiles/colormanagement: config.ocio
 * and luts/) whose Filmic LUTs (filmic_desat65cube.spi3d,
 * filmic_to_0-70_1-03.spi1d) implement RR_VIEW_FILMIC on ctx. NULL or "":
 * no LUTs (Filmic frames fall back to Standard, flagged). rr_create reads
 * the RR_OCIO_DIR environment variable the same way. RR_ENOENT / RR_EINVAL
 * if the LUT files are missing or malformed (ctx keeps no LUTs then). */
int rr_set_ocio_config(rr_ctx* ctx, const char* dir);

void rr_scene_free(rr_scene* scene);
void rr_destroy(rr_ctx* ctx);

/* ------------------------------------------------------------------------ *
 * Inspection entry points. Not on the production path; they expose the
 * intermediate state of a frame so the parity tests (tests/) can compare every
 * stage with the CPU oracle (oracle/) on identical inputs.
 * ------------------------------------------------------------------------ */

#define RR_CAM_FLOATS 16   /* pos3 right3 up3 back3 half_w half_h clip_start clip_end */
#define RR_LIGHT_FLOATS 12 /* type pos3 dir3 radius intensity3 pad */
#define RR_MAT_FLOATS 12   /* base3 metallic specular roughness ior emission3 model pad */
#define RR_RENDER_INTS 10  /* W H spp max_bounces seed view_transform spp_per_chunk bvh_width
                              max_diffuse_bounces max_glossy_bounces */
#define RR_RENDER_FLOATS 4 /* clamp_indirect filter_width exposure_scale pad */

int rr_debug_counts(rr_scene* scene, int32_t* n_triangles, int32_t* n_lights,
                    int32_t* n_materials, int32_t* n_objects);

/* The scene's triangles in object space as loaded (generators expanded):
 * tri_local9 n*9 floats (v0 v1 v2), tri_object n object indices (the matrix
 * of rr_debug_object_matrix that places it). Either pointer may be NULL.
 * Test infrastructure: pins the device's world transform (k_transform)
 * against a host restatement; no reference counterpart. */
int rr_debug_scene_mesh(rr_scene* scene, float* tri_local9, int32_t* tri_object);

/* Evaluate the frame on the device (animation, world transform, LBVH) and read
 * back what the integrator consumes. Any output pointer may be NULL. */
int rr_debug_frame_state(rr_ctx* ctx, rr_scene* scene, int32_t frame_index,
                         const rr_render_params* params, float* tris_world /* n*9 */,
                         int32_t* tri_material /* n */, float* camera /* RR_CAM_FLOATS */,
                         float* lights /* n_lights*RR_LIGHT_FLOATS */,
                         float* materials /* n_mat*RR_MAT_FLOATS */, float* world /* 3 */,
                         int32_t* render_ints /* RR_RENDER_INTS */,
                         float* render_floats /* RR_RENDER_FLOATS */);

/* Hierarchy of the frame (rr_debug_bvh_hier): sorted Morton keys and primitive order (n each), internal
 * node children (2*(n-1); leaf = ~sorted_index) and child boxes (12*(n-1):
 * lmin3 lmax3 rmin3 rmax3). n == 1 yields one root whose two children are leaf 0. */
int rr_debug_bvh(rr_ctx* ctx, rr_scene* scene, int32_t frame_index, uint32_t* keys,
                 uint32_t* order, int32_t* children, float* boxes);

/* rr_debug_bvh of a chosen hierarchy: hier 2 = Karras LBVH, 3 = PLOC, 0 = the
 * one the frame kernels use (what rr_debug_bvh returns). */
int rr_debug_bvh_hier(rr_ctx* ctx, rr_scene* scene, int32_t frame_index, int32_t hier, uint32_t* keys,
                      uint32_t* order, int32_t* children, float* boxes);

/* Quantised 6-wide hierarchy of the frame (the PLOC hierarchy collapsed into
 * 6-wide nodes, the hierarchy the split path of large scenes traverses; built
 * on demand here). *nq receives the node count; if children / nodes16 are
 * non-NULL they receive 6*nq child refs (>= 0 node, < 0 ~position in the
 * hierarchy's triangle array, 0x7fffffff unused slot — spelled out from the
 * node's implicit references) and the 16 32-bit words of each 64-byte node:
 * origin x y z (float), exponent bytes (e+128 per axis) | internal-slot mask
 * << 24, first internal child, first leaf triangle, lo x / lo y / lo z / hi x /
 * hi y / hi z grid coordinates of children 0..3 (one byte each), children 4
 * and 5 as byte pairs (lo x, lo y), (lo z, hi x), (hi y, hi z), one zero word;
 * tri_orig (n triangles) the original triangle id at each position of that
 * array. Call once with NULL arrays to size them. */
int rr_debug_qbvh(rr_ctx* ctx, rr_scene* scene, int32_t frame_index, int32_t* nq,
                  int32_t* children, uint32_t* nodes16, int32_t* tri_orig);

/* Trace a batch of rays against the frame's hierarchy. bvh_width: 2 (LBVH),
 * 4 (the quantised 6-wide collapse), 5 (the same hierarchy walked by the camera
 * kernel's 64-ray packets, with 4 packet-stack entries in LDS so that the
 * stack's HBM part is used; closest hit only, occluded = 255), 6 (the
 * 6-wide per-lane walk with one LDS stack entry per lane, so that its grouped
 * entries live in the HBM part), 7 (the camera kernel's default packet walk,
 * one box test per child for the whole packet — packet_trace_beam — with the
 * same 4-entry LDS stack as 5; exact only for packets whose rays share one
 * origin, as camera rays do; closest hit only) or 0 (whichever
 * the frame kernels use for this scene, render_ints[7] of rr_debug_frame_state). rays: n*8 floats
 * (o.xyz, tmin, d.xyz, tmax). hits: n*4 floats (t, u, v, 0), prims: n original
 * triangle ids (-1 miss), occluded: n bytes (any-hit result). */
int rr_debug_trace(rr_ctx* ctx, rr_scene* scene, int32_t frame_index, int32_t bvh_width,
                   int32_t n_rays, const float* rays, float* hits, int32_t* prims,
                   uint8_t* occluded);

/* BSDF sampling at one shading point, as the frame kernels sample it: the
 * material (RR_MAT_FLOATS, rr_debug_frame_state layout), unit normal n3 and
 * view direction wo3; per draw i the three numbers u[3i..3i+2] (lobe pick,
 * disk u1, u2). Outputs per draw: wi3, f3 (BSDF value), pdf and ok (0 the
 * path ends, 1 diffuse lobe, 2 glossy lobe). */
int rr_debug_bsdf_sample(rr_ctx* ctx, const float* mat12, const float* n3, const float* wo3, int32_t n,
                         const float* u, float* wi3, float* f3, float* pdf, int32_t* ok);

/* The tile kernel's scheduling record of the last frame enqueued (LDS-resident
 * scenes): per screen tile (8x8 pixels, row-major), the real-time ticks
 * (100 MHz) its work units took in that frame's k_tiles launch (0 for tiles
 * outside the scene's screen box), and the box tiles' hand-out order that
 * launch used (built from the launch before it; its first entries are the
 * box tiles). Up to `capacity` entries of each; *n_tiles = the length of the
 * slot's buffers (at least the frame's tile count; 0: no tile frame yet).
 * unit_log (may be null): when that frame was rendered with
 * RR_FLAG_COUNT_TRAVERSAL, per box work unit u (hand-out number, below
 * unit_capacity and 65536) its start and end real-time ticks (2 per unit;
 * 0, 0: not logged). */
int rr_debug_tile_costs(rr_ctx* ctx, int32_t capacity, uint32_t* costs, int32_t* order, int32_t* n_tiles,
                        uint64_t* unit_log, int32_t unit_capacity);

/* The per-sample path's square roots and reciprocals (rr_device.h sqrt_rn /
 * sqrt_any / rcp_rn) against the device's correctly rounded sqrtf and
 * 1.0f / x, over the float bit patterns lo .. lo + n - 1: counts5[0] =
 * sqrt_rn mismatches with the argument in its range (+-0 or [2^-96, FLT_MAX];
 * must be 0), [1] = sqrt_rn mismatches outside it (not called there), [2] =
 * sqrt_any mismatches (must be 0), [3] = rcp_rn mismatches with |x| in
 * [2^-126, 2^126) (must be 0), [4] = rcp_rn mismatches outside it. Test
 * infrastructure for the bit-exactness claim; no reference counterpart. */
int rr_debug_fastmath_check(rr_ctx* ctx, uint32_t lo, uint64_t n, uint64_t* counts5);

/* Host animation evaluation: object_to_world matrix (row-major 4x4, f64) of
 * object `object_index` at (possibly fractional) frame. */
int rr_debug_object_matrix(rr_scene* scene, int32_t object_index, double frame,
                           double* m16);

#ifdef __cplusplus
}
#endif

#endif /* RR_H */
