"""ctypes binding of the renderer's C ABI (include/rr.h, lib/librr.so).

This is the Python host's view of the drop-in boundary; the Rust worker binds
the same symbols through an `extern "C"` block. The library is
the in-tree build from __graft_entry__.build(); there is no fallback: if it is
missing or fails to load, every entry point raises RRError.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "librr.so")
SHIM_PATH = os.path.join(_HERE, "lib", "rr-blender-shim")

RR_OK, RR_ENOENT, RR_EIO, RR_ENOMEM, RR_ENODEV, RR_EINVAL, RR_ENOTSUP = 0, -2, -5, -12, -19, -22, -95
RR_EBUSY = -16
RR_MAX_FRAMES_IN_FLIGHT = 3
RR_VIEW_SCENE, RR_VIEW_STANDARD, RR_VIEW_RAW, RR_VIEW_FILMIC = -1, 0, 1, 2
RR_ABI_VERSION = 8
QWIDTH = 6  # children per quantised node of the split path (rr_device.h kQWidth)
RR_CAM_FLOATS, RR_LIGHT_FLOATS, RR_MAT_FLOATS, RR_RENDER_INTS, RR_RENDER_FLOATS = 16, 12, 12, 10, 4


class RRError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"rr error {code}: {message}")
        self.code = code


class RenderParams(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int32), ("max_bounces", ctypes.c_int32),
                ("clamp_indirect", ctypes.c_float), ("seed", ctypes.c_uint32),
                ("use_scene_seed", ctypes.c_int32), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("view_transform", ctypes.c_int32),
                ("spp_per_chunk", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("max_diffuse_bounces", ctypes.c_int32), ("max_glossy_bounces", ctypes.c_int32)]


class FrameTiming(ctypes.Structure):
    _fields_ = [("loaded_at", ctypes.c_double), ("started_rendering_at", ctypes.c_double),
                ("finished_rendering_at", ctypes.c_double), ("file_saving_started_at", ctypes.c_double),
                ("file_saving_finished_at", ctypes.c_double)]


class FrameStats(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("chunks", ctypes.c_int32), ("camera_rays", ctypes.c_uint64),
                ("extension_rays", ctypes.c_uint64), ("shadow_rays", ctypes.c_uint64),
                ("primary_continued", ctypes.c_uint64), ("primary_shadow", ctypes.c_uint64),
                ("anim_ms", ctypes.c_double), ("build_ms", ctypes.c_double), ("trace_ms", ctypes.c_double),
                ("readback_ms", ctypes.c_double), ("encode_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("bvh_rebuilt", ctypes.c_int32), ("n_triangles", ctypes.c_int32),
                ("output_bytes", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double * 8), ("kernel_launches", ctypes.c_int32 * 8),
                ("trav_nodes", ctypes.c_uint64 * 3), ("trav_tris", ctypes.c_uint64 * 3),
                ("camera_rays_traced", ctypes.c_uint64), ("view_transform", ctypes.c_int32),
                ("view_transform_substituted", ctypes.c_int32), ("kernel_clock_ghz", ctypes.c_double),
                ("kernel_wave_fill", ctypes.c_double), ("tile_slices", ctypes.c_int32),
                ("stack_drops", ctypes.c_int32),
                ("extension_rays_escaped", ctypes.c_uint64), ("shadow_rays_escaped", ctypes.c_uint64),
                ("kernel_entry_spread", ctypes.c_double), ("kernel_exit_spread", ctypes.c_double)]

    def as_dict(self) -> dict:
        out = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            out[k] = list(v) if not isinstance(v, (int, float)) else v
        return out


RR_FLAG_PROFILE_KERNELS, RR_FLAG_COUNT_TRAVERSAL, RR_FLAG_WAVEFRONT = 1, 2, 4
KERNEL_CLASSES = ["build", "primary", "extend", "shadow", "accumulate", "shade", "tiles"]


# Every symbol include/rr.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "rr_render_params_default", "rr_abi_version", "rr_create", "rr_scene_load", "rr_render_frame",
    "rr_frame_submit", "rr_frame_complete",
    "rr_render_frame_to_memory", "rr_scene_resolution", "rr_encode_image", "rr_last_error",
    "rr_last_warning", "rr_set_ocio_config", "rr_synchronize",
    "rr_scene_free", "rr_destroy", "rr_debug_counts", "rr_debug_scene_mesh", "rr_debug_frame_state", "rr_debug_bvh",
    "rr_debug_trace", "rr_debug_object_matrix", "rr_debug_qbvh", "rr_debug_bvh_hier", "rr_debug_jpeg_device",
    "rr_debug_bsdf_sample", "rr_debug_fastmath_check", "rr_debug_tile_costs",
]

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # RR_LIB_PATH: an alternative in-tree build of the same library (A/B timing
    # of kernel variants, tools/ab_variants.sh); never a different implementation.
    path = os.environ.get("RR_LIB_PATH", LIB_PATH)
    if not os.path.isfile(path):
        raise RRError(RR_ENOENT, f"{path} is missing: build it with __graft_entry__.build() "
                                 "(there is no CPU fallback)")
    L = ctypes.CDLL(path)
    if L.rr_abi_version() != RR_ABI_VERSION:
        raise RRError(RR_EINVAL, f"{path}: ABI {L.rr_abi_version()}, this binding expects {RR_ABI_VERSION} "
                                 "(rebuild with __graft_entry__.build())")
    P, c_int, i32, u32, f32p, u8p = ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_uint32, \
        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint8)
    i32p, u32p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint32)
    sig = {
        "rr_render_params_default": (None, [ctypes.POINTER(RenderParams)]),
        "rr_abi_version": (i32, []),
        "rr_create": (c_int, [c_int, ctypes.POINTER(P)]),
        "rr_scene_load": (c_int, [P, ctypes.c_char_p, ctypes.POINTER(P)]),
        "rr_render_frame": (c_int, [P, P, i32, ctypes.POINTER(RenderParams), ctypes.c_char_p, ctypes.c_char_p, i32,
                                    ctypes.POINTER(FrameTiming), ctypes.POINTER(FrameStats)]),
        "rr_frame_submit": (c_int, [P, P, i32, ctypes.POINTER(RenderParams), ctypes.c_char_p, ctypes.c_char_p, i32,
                                    ctypes.POINTER(ctypes.c_uint64)]),
        "rr_frame_complete": (c_int, [P, ctypes.c_uint64, ctypes.POINTER(FrameTiming), ctypes.POINTER(FrameStats)]),
        "rr_render_frame_to_memory": (c_int, [P, P, i32, ctypes.POINTER(RenderParams), f32p, u8p,
                                              ctypes.POINTER(FrameStats)]),
        "rr_scene_resolution": (c_int, [P, ctypes.POINTER(RenderParams), i32p, i32p]),
        "rr_encode_image": (c_int, [u8p, i32, i32, ctypes.c_char_p, ctypes.c_char_p, i32,
                                    ctypes.POINTER(ctypes.c_uint64)]),
        "rr_last_error": (ctypes.c_char_p, [P]),
        "rr_last_warning": (ctypes.c_char_p, [P]),
        "rr_set_ocio_config": (c_int, [P, ctypes.c_char_p]),
        "rr_synchronize": (c_int, [P]),
        "rr_scene_free": (None, [P]),
        "rr_destroy": (None, [P]),
        "rr_debug_counts": (c_int, [P, i32p, i32p, i32p, i32p]),
        "rr_debug_scene_mesh": (c_int, [P, f32p, i32p]),
        "rr_debug_frame_state": (c_int, [P, P, i32, ctypes.POINTER(RenderParams), f32p, i32p, f32p, f32p, f32p,
                                         f32p, i32p, f32p]),
        "rr_debug_bvh": (c_int, [P, P, i32, u32p, u32p, i32p, f32p]),
        "rr_debug_trace": (c_int, [P, P, i32, i32, i32, f32p, f32p, i32p, u8p]),
        "rr_debug_qbvh": (c_int, [P, P, i32, i32p, i32p, u32p, i32p]),
        "rr_debug_bvh_hier": (c_int, [P, P, i32, i32, u32p, u32p, i32p, f32p]),
        "rr_debug_jpeg_device": (c_int, [P, u8p, i32, i32, i32, u8p, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_uint64)]),
        "rr_debug_object_matrix": (c_int, [P, i32, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
        "rr_debug_bsdf_sample": (c_int, [P, f32p, f32p, f32p, i32, f32p, f32p, f32p, f32p, i32p]),
        "rr_debug_fastmath_check": (c_int, [P, ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
        "rr_debug_tile_costs": (c_int, [P, c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64), c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int, ctx=None):
    if rc != 0:
        msg = lib().rr_last_error(ctx).decode("utf-8", "replace")
        raise RRError(rc, msg)


def _ptr(a: np.ndarray | None, ctype):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def default_params(**overrides) -> RenderParams:
    p = RenderParams()
    lib().rr_render_params_default(ctypes.byref(p))
    for k, v in overrides.items():
        if v is None:
            continue
        if k == "seed":
            p.use_scene_seed = 0
        setattr(p, k, v)
    return p


@dataclass
class FrameState:
    tris: np.ndarray        # (n, 3, 3) world-space vertices
    tri_mat: np.ndarray     # (n,)
    camera: np.ndarray      # (16,)
    lights: np.ndarray      # (nl, 12)
    materials: np.ndarray   # (nm, 12)
    world: np.ndarray       # (3,)
    render_ints: np.ndarray  # (RR_RENDER_INTS,)
    render_floats: np.ndarray  # (4,)


class Scene:
    """An exported project (.rrscene) — host-only until a RenderContext uses it."""

    def __init__(self, path: str, ctx: "RenderContext | None" = None):
        self.path = os.fspath(path)
        h = ctypes.c_void_p()
        _check(lib().rr_scene_load(ctx.handle if ctx else None, self.path.encode(), ctypes.byref(h)))
        self.handle = h
        self.ctx = ctx

    def close(self):
        if self.handle:
            lib().rr_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def counts(self) -> dict:
        v = [ctypes.c_int32() for _ in range(4)]
        _check(lib().rr_debug_counts(self.handle, *[ctypes.byref(x) for x in v]))
        return dict(zip(["triangles", "lights", "materials", "objects"], [x.value for x in v]))

    def mesh(self) -> tuple[np.ndarray, np.ndarray]:
        """Object-space triangles (n, 3, 3) float32 and the object index of each
        (rr_debug_scene_mesh)."""
        n = self.counts()["triangles"]
        local = np.zeros((max(n, 1), 3, 3), np.float32)
        obj = np.zeros(max(n, 1), np.int32)
        _check(lib().rr_debug_scene_mesh(self.handle, _ptr(local, ctypes.c_float), _ptr(obj, ctypes.c_int32)))
        return local[:n], obj[:n]

    def resolution(self, params: RenderParams | None = None) -> tuple[int, int]:
        w, h = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().rr_scene_resolution(self.handle, ctypes.byref(params) if params else None,
                                         ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def frame_constants(self, frame: int, params: RenderParams | None = None) -> FrameState:
        """Host-only frame evaluation (no device): camera, lights, materials, world, render ints/floats."""
        c = self.counts()
        nl, nm = c["lights"], c["materials"]
        cam = np.zeros(RR_CAM_FLOATS, np.float32)
        lights = np.zeros((max(nl, 1), RR_LIGHT_FLOATS), np.float32)
        mats = np.zeros((max(nm, 1), RR_MAT_FLOATS), np.float32)
        world = np.zeros(3, np.float32)
        ri = np.zeros(RR_RENDER_INTS, np.int32)
        rf = np.zeros(RR_RENDER_FLOATS, np.float32)
        tm = np.zeros(max(c["triangles"], 1), np.int32)
        _check(lib().rr_debug_frame_state(None, self.handle, int(frame), ctypes.byref(params) if params else None,
                                          None, _ptr(tm, ctypes.c_int32), _ptr(cam, ctypes.c_float),
                                          _ptr(lights, ctypes.c_float),
                                          _ptr(mats, ctypes.c_float), _ptr(world, ctypes.c_float),
                                          _ptr(ri, ctypes.c_int32), _ptr(rf, ctypes.c_float)))
        # tris stay empty (world triangles need the device); tri_mat is the scene's, per triangle
        return FrameState(np.zeros((0, 3, 3), np.float32), tm[:c["triangles"]], cam, lights[:nl], mats[:nm],
                          world, ri, rf)

    def object_matrix(self, obj: int, frame: float) -> np.ndarray:
        m = (ctypes.c_double * 16)()
        _check(lib().rr_debug_object_matrix(self.handle, obj, float(frame), m))
        return np.array(m[:], dtype=np.float64).reshape(4, 4)


class RenderContext:
    """One HIP device (rr_ctx). Not thread-safe; one frame in flight at a time."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().rr_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            lib().rr_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def load_scene(self, path: str) -> Scene:
        return Scene(path, self)

    def set_ocio_config(self, directory: str | None):
        """rr_set_ocio_config: Blender colour-management directory whose Filmic
        LUTs implement RR_VIEW_FILMIC (None: none; Filmic falls back to Standard)."""
        _check(lib().rr_set_ocio_config(self.handle, directory.encode() if directory else None), self.handle)

    def synchronize(self):
        """rr_synchronize: wait for all device work this context enqueued."""
        _check(lib().rr_synchronize(self.handle), self.handle)

    def last_warning(self) -> str:
        return lib().rr_last_warning(self.handle).decode("utf-8", "replace")

    def render_frame(self, scene: Scene, frame: int, params: RenderParams | None = None,
                     out_path: str | None = None, fmt: str | None = "JPEG", quality: int = 90):
        t, s = FrameTiming(), FrameStats()
        _check(lib().rr_render_frame(self.handle, scene.handle, int(frame),
                                     ctypes.byref(params) if params else None,
                                     out_path.encode() if out_path is not None else None,
                                     fmt.encode() if (fmt is not None and out_path is not None) else None,
                                     int(quality), ctypes.byref(t), ctypes.byref(s)), self.handle)
        return t, s

    def submit_frame(self, scene: Scene, frame: int, params: RenderParams | None = None,
                     out_path: str | None = None, fmt: str | None = "JPEG", quality: int = 90) -> int:
        """rr_frame_submit: enqueue the frame's device work, return its ticket."""
        t = ctypes.c_uint64()
        _check(lib().rr_frame_submit(self.handle, scene.handle, int(frame),
                                     ctypes.byref(params) if params else None,
                                     out_path.encode() if out_path is not None else None,
                                     fmt.encode() if (fmt is not None and out_path is not None) else None,
                                     int(quality), ctypes.byref(t)), self.handle)
        return int(t.value)

    def complete_frame(self, ticket: int):
        """rr_frame_complete: wait, encode + write; (timing, stats)."""
        t, s = FrameTiming(), FrameStats()
        _check(lib().rr_frame_complete(self.handle, ctypes.c_uint64(ticket), ctypes.byref(t), ctypes.byref(s)),
               self.handle)
        return t, s

    def render_to_memory(self, scene: Scene, frame: int, params: RenderParams | None = None,
                         film: bool = True, rgba: bool = True):
        w, h = scene.resolution(params)
        f = np.zeros((h, w, 4), np.float32) if film else None
        r = np.zeros((h, w, 4), np.uint8) if rgba else None
        s = FrameStats()
        _check(lib().rr_render_frame_to_memory(self.handle, scene.handle, int(frame),
                                               ctypes.byref(params) if params else None,
                                               _ptr(f, ctypes.c_float), _ptr(r, ctypes.c_uint8),
                                               ctypes.byref(s)), self.handle)
        return f, r, s

    def frame_state(self, scene: Scene, frame: int, params: RenderParams | None = None) -> FrameState:
        c = scene.counts()
        n, nl, nm = c["triangles"], c["lights"], c["materials"]
        tris = np.zeros((max(n, 1), 3, 3), np.float32)
        mats_i = np.zeros(max(n, 1), np.int32)
        cam = np.zeros(RR_CAM_FLOATS, np.float32)
        lights = np.zeros((max(nl, 1), RR_LIGHT_FLOATS), np.float32)
        mats = np.zeros((max(nm, 1), RR_MAT_FLOATS), np.float32)
        world = np.zeros(3, np.float32)
        ri = np.zeros(RR_RENDER_INTS, np.int32)
        rf = np.zeros(RR_RENDER_FLOATS, np.float32)
        _check(lib().rr_debug_frame_state(self.handle, scene.handle, int(frame),
                                          ctypes.byref(params) if params else None,
                                          _ptr(tris, ctypes.c_float) if self.handle else None,
                                          _ptr(mats_i, ctypes.c_int32),
                                          _ptr(cam, ctypes.c_float), _ptr(lights, ctypes.c_float),
                                          _ptr(mats, ctypes.c_float), _ptr(world, ctypes.c_float),
                                          _ptr(ri, ctypes.c_int32), _ptr(rf, ctypes.c_float)), self.handle)
        return FrameState(tris[:n], mats_i[:n], cam, lights[:nl], mats[:nm], world, ri, rf)

    def bvh(self, scene: Scene, frame: int, hier: int = 0):
        """rr_debug_bvh_hier: (keys, order, children (ni,2), boxes (ni,12)); hier
        2 = LBVH, 3 = PLOC, 0 = the frame's hierarchy."""
        n = scene.counts()["triangles"]
        ni = max(n - 1, 1)
        keys = np.zeros(n, np.uint32)
        order = np.zeros(n, np.uint32)
        children = np.zeros((ni, 2), np.int32)
        boxes = np.zeros((ni, 12), np.float32)
        _check(lib().rr_debug_bvh_hier(self.handle, scene.handle, int(frame), int(hier), _ptr(keys, ctypes.c_uint32),
                                  _ptr(order, ctypes.c_uint32), _ptr(children, ctypes.c_int32),
                                  _ptr(boxes, ctypes.c_float)), self.handle)
        return keys, order, children, boxes

    def qbvh(self, scene: Scene, frame: int, with_order: bool = False):
        """rr_debug_qbvh: (children (nq, QWIDTH) with the implicit references
        spelled out, nodes (nq, 16) uint32: the raw 64-byte quantised nodes,
        rr_device.h QNode6); with_order: also the original triangle id at each
        position of the hierarchy's triangle array."""
        nq = ctypes.c_int32()
        _check(lib().rr_debug_qbvh(self.handle, scene.handle, int(frame), ctypes.byref(nq), None, None, None),
               self.handle)
        ch = np.zeros((max(nq.value, 1), QWIDTH), np.int32)
        bx = np.zeros((max(nq.value, 1), 16), np.uint32)
        orig = np.zeros(max(scene.counts()["triangles"], 1), np.int32)
        _check(lib().rr_debug_qbvh(self.handle, scene.handle, int(frame), ctypes.byref(nq), _ptr(ch, ctypes.c_int32),
                                   _ptr(bx, ctypes.c_uint32), _ptr(orig, ctypes.c_int32)), self.handle)
        if with_order:
            return ch[:nq.value], bx[:nq.value], orig[:scene.counts()["triangles"]]
        return ch[:nq.value], bx[:nq.value]

    def jpeg_device(self, rgba: np.ndarray, quality: int = 90) -> bytes:
        """rr_debug_jpeg_device: the JPEG file bytes of an (H, W, 4) uint8 image
        encoded on the device (forward DCT + Huffman coding)."""
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        h, w = rgba.shape[:2]
        n = ctypes.c_uint64()
        _check(lib().rr_debug_jpeg_device(self.handle, _ptr(rgba, ctypes.c_uint8), w, h, int(quality), None, 0,
                                          ctypes.byref(n)), self.handle)
        out = np.zeros(n.value, np.uint8)
        _check(lib().rr_debug_jpeg_device(self.handle, _ptr(rgba, ctypes.c_uint8), w, h, int(quality),
                                          _ptr(out, ctypes.c_uint8), n.value, ctypes.byref(n)), self.handle)
        return out.tobytes()

    def bsdf_sample(self, mat12, n, wo, u):
        """rr_debug_bsdf_sample: (wi [k,3], f [k,3], pdf [k], ok [k]: 0 end, 1 diffuse, 2 glossy)."""
        f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
        m, n, wo, u = f32(mat12), f32(n), f32(wo), f32(u).reshape(-1, 3)
        k = u.shape[0]
        wi, f = np.zeros((k, 3), np.float32), np.zeros((k, 3), np.float32)
        pdf, ok = np.zeros(k, np.float32), np.zeros(k, np.int32)
        _check(lib().rr_debug_bsdf_sample(self.handle, _ptr(m, ctypes.c_float), _ptr(n, ctypes.c_float),
                                          _ptr(wo, ctypes.c_float), k, _ptr(u, ctypes.c_float),
                                          _ptr(wi, ctypes.c_float), _ptr(f, ctypes.c_float),
                                          _ptr(pdf, ctypes.c_float), _ptr(ok, ctypes.c_int32)), self.handle)
        return wi, f, pdf, ok

    def fastmath_check(self, lo: int = 0, n: int = 1 << 32):
        """rr_debug_fastmath_check: mismatches of (sqrt_rn in range, sqrt_rn outside, sqrt_any,
        rcp_rn in range, rcp_rn outside)."""
        out = (ctypes.c_uint64 * 5)()
        _check(lib().rr_debug_fastmath_check(self.handle, int(lo), int(n), out), self.handle)
        return tuple(int(v) for v in out)

    def tile_costs(self, capacity: int = 1 << 20, units: int = 1 << 16):
        """rr_debug_tile_costs: (per-tile real-time ticks of the last tile frame's
        units, the box tiles' hand-out order it used, each of the slot buffers'
        length; per box unit u its (start, end) ticks when that frame was a
        counting frame, shape (units, 2))."""
        costs = np.zeros(capacity, np.uint32)
        order = np.zeros(capacity, np.int32)
        log = np.zeros((max(units, 1), 2), np.uint64)
        n = ctypes.c_int32(0)
        _check(lib().rr_debug_tile_costs(self.handle, capacity, _ptr(costs, ctypes.c_uint32),
                                         _ptr(order, ctypes.c_int32), ctypes.byref(n),
                                         _ptr(log, ctypes.c_uint64), units), self.handle)
        m = min(int(n.value), capacity)
        return costs[:m], order[:m], log[:units]

    def trace(self, scene: Scene, frame: int, rays: np.ndarray, width: int = 0):
        """rr_debug_trace; width 0 = the hierarchy the frame kernels use."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = rays.shape[0]
        hits = np.zeros((max(n, 1), 4), np.float32)
        prims = np.zeros(max(n, 1), np.int32)
        occ = np.zeros(max(n, 1), np.uint8)
        _check(lib().rr_debug_trace(self.handle, scene.handle, int(frame), int(width), n, _ptr(rays, ctypes.c_float),
                                    _ptr(hits, ctypes.c_float), _ptr(prims, ctypes.c_int32),
                                    _ptr(occ, ctypes.c_uint8)), self.handle)
        return hits[:n], prims[:n], occ[:n]


def encode_image(rgba: np.ndarray, out_path_no_ext: str, fmt: str, quality: int = 90) -> int:
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = rgba.shape[:2]
    nbytes = ctypes.c_uint64()
    _check(lib().rr_encode_image(_ptr(rgba, ctypes.c_uint8), w, h, out_path_no_ext.encode(), fmt.encode(),
                                 int(quality), ctypes.byref(nbytes)))
    return nbytes.value
