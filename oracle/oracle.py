"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the CPU oracle (rr_oracle.c).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker. The product (the package's native.py / librr.so) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
QW = 6  # child slots per quantised wide node (rr_oracle.c ORC_QW_MAX, rr_device.h kQWidth)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB):
            build()
        L = ctypes.CDLL(LIB)
        f, i32, u32, u8 = (ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint8))
        c_int = ctypes.c_int
        L.orc_build_lbvh.argtypes = [c_int, f, u32, u32, i32, f]
        L.orc_build_bvh.argtypes = [c_int, f, c_int, u32, u32, i32, f]
        L.orc_trace.argtypes = [c_int, f, c_int, f, f, i32, u8]
        L.orc_trace_w.argtypes = [c_int, f, c_int, c_int, f, f, i32, u8]
        L.orc_build_qbvh.argtypes = [c_int, f, i32, i32, u32, i32]
        L.orc_trace_brute.argtypes = [c_int, f, c_int, f, f, i32]
        L.orc_render.argtypes = [c_int, f, i32, f, c_int, f, f, f, i32, f, f, u8, c_int, c_int, c_int]
        L.orc_rng.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, c_int, f]
        L.orc_disk.argtypes = [c_int, f, f]
        L.orc_bsdf_eval.argtypes = [f, f, f, f, f, f]
        L.orc_bsdf_eval_n.argtypes = [f, f, f, c_int, f, f, f]
        L.orc_bsdf_sample.argtypes = [f, f, f, c_int, f, f, f, f, i32]
        L.orc_filter_table.argtypes = [ctypes.c_float, f]
        L.orc_srgb_lut.argtypes = [f]
        L.orc_material_lut.argtypes = [f, f]
        L.orc_set_filmic.argtypes = [f, c_int, f, c_int, c_int, ctypes.c_float, ctypes.c_float]
        L.orc_filmic.argtypes = [c_int, f, u8]
        L.orc_set_rules.argtypes = [c_int, c_int]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(t))


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def build_lbvh(tris: np.ndarray, hier: int = 2):
    """Sorted keys, order, children and child boxes of the hierarchy `hier`
    (2 = Karras LBVH, 3 = PLOC) as rr_debug_bvh."""
    tris = _f32(tris).reshape(-1, 9)
    n = tris.shape[0]
    ni = max(n - 1, 1)
    keys, order = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    children, boxes = np.zeros((ni, 2), np.int32), np.zeros((ni, 12), np.float32)
    lib().orc_build_bvh(n, _p(tris, ctypes.c_float), int(hier), _p(keys, ctypes.c_uint32),
                        _p(order, ctypes.c_uint32), _p(children, ctypes.c_int32), _p(boxes, ctypes.c_float))
    return keys, order, children, boxes


def trace(tris: np.ndarray, rays: np.ndarray, width: int = 2):
    """Closest + any hit through the LBVH (2), PLOC (3) or PLOC's quantised 6-wide collapse (4)."""
    tris = _f32(tris).reshape(-1, 9)
    rays = _f32(rays).reshape(-1, 8)
    n = rays.shape[0]
    hits, prims, occ = np.zeros((n, 4), np.float32), np.zeros(n, np.int32), np.zeros(n, np.uint8)
    lib().orc_trace_w(tris.shape[0], _p(tris, ctypes.c_float), int(width), n, _p(rays, ctypes.c_float),
                      _p(hits, ctypes.c_float), _p(prims, ctypes.c_int32), _p(occ, ctypes.c_uint8))
    return hits, prims, occ


def build_qbvh(tris: np.ndarray, with_order: bool = False):
    """Quantised 6-wide hierarchy: (children (n, QW), nodes (n, 16) uint32) as rr_debug_qbvh;
    with_order: also the original triangle id of each position of the BVH4's
    triangle array (the order its leaf ranges index)."""
    tris = _f32(tris).reshape(-1, 9)
    n = tris.shape[0]
    ni = max(n - 1, 1)
    n4 = np.zeros(1, np.int32)
    ch, bx = np.zeros((ni, QW), np.int32), np.zeros((ni, 16), np.uint32)
    orig = np.zeros(max(n, 1), np.int32)
    lib().orc_build_qbvh(n, _p(tris, ctypes.c_float), _p(n4, ctypes.c_int32), _p(ch, ctypes.c_int32),
                         _p(bx, ctypes.c_uint32), _p(orig, ctypes.c_int32))
    if with_order:
        return ch[:n4[0]], bx[:n4[0]], orig[:n]
    return ch[:n4[0]], bx[:n4[0]]


def trace_brute(tris: np.ndarray, rays: np.ndarray):
    tris = _f32(tris).reshape(-1, 9)
    rays = _f32(rays).reshape(-1, 8)
    n = rays.shape[0]
    hits, prims = np.zeros((n, 4), np.float32), np.zeros(n, np.int32)
    lib().orc_trace_brute(tris.shape[0], _p(tris, ctypes.c_float), n, _p(rays, ctypes.c_float),
                          _p(hits, ctypes.c_float), _p(prims, ctypes.c_int32))
    return hits, prims


def render(tris, tri_mat, camera, lights, materials, world, render_ints, render_floats,
           rows: tuple[int, int] | None = None, threads: int = 0, film: bool = True, rgba: bool = True,
           row_list=None):
    """Full-frame render of the oracle path tracer. Inputs as rr_debug_frame_state.
    rows: a range of rows; row_list: any rows (one hierarchy build for all)."""
    tris = _f32(tris).reshape(-1, 9)
    tri_mat = np.ascontiguousarray(tri_mat, dtype=np.int32)
    cam = _f32(camera)
    lights = _f32(lights).reshape(-1, 12)
    mats = _f32(materials).reshape(-1, 12)
    world = _f32(world)
    ri = np.asarray(render_ints, dtype=np.int32)
    if ri.size < 10:  # per-lobe bounce caps default to Cycles' 4 / 4 (rr.h render_ints[8], [9])
        ri = np.concatenate([ri, np.array([4, 4], np.int32)[: 10 - ri.size]])
    ri = np.ascontiguousarray(ri)
    rf = _f32(render_floats)
    W, H = int(ri[0]), int(ri[1])
    f = np.zeros((H, W, 4), np.float32) if film else None
    r = np.zeros((H, W, 4), np.uint8) if rgba else None
    r0, r1 = rows if rows else (0, 0)
    rl = None
    if row_list is not None:
        rl = np.ascontiguousarray(row_list, dtype=np.int32)
        assert rl.size > 0 and rl.min() >= 0 and rl.max() < H
        lib().orc_set_row_list(_p(rl, ctypes.c_int32), int(rl.size))
    try:
        _render_call(tris, tri_mat, cam, lights, mats, world, ri, rf, f, r, r0, r1, threads)
    finally:
        if rl is not None:
            lib().orc_set_row_list(None, 0)
    return f, r


def _render_call(tris, tri_mat, cam, lights, mats, world, ri, rf, f, r, r0, r1, threads):
    lib().orc_render(tris.shape[0], _p(tris, ctypes.c_float), _p(tri_mat, ctypes.c_int32), _p(cam, ctypes.c_float),
                     lights.shape[0], _p(lights, ctypes.c_float), _p(mats, ctypes.c_float),
                     _p(world, ctypes.c_float), _p(ri, ctypes.c_int32), _p(rf, ctypes.c_float),
                     _p(f, ctypes.c_float), _p(r, ctypes.c_uint8), r0, r1, threads)


class rules:
    """Context manager: orc_render's shortcuts switched for a block (test use),
    e.g. `with O.rules(cull=False): ...`. Both are restored to on afterwards."""

    def __init__(self, cull: bool = True, hull: bool = True):
        self.cull, self.hull = cull, hull

    def __enter__(self):
        lib().orc_set_rules(int(self.cull), int(self.hull))
        return self

    def __exit__(self, *exc):
        lib().orc_set_rules(1, 1)
        return False


def render_state(state, **kw):
    """Render from a product FrameState (native.RenderContext.frame_state)."""
    return render(state.tris, state.tri_mat, state.camera, state.lights, state.materials, state.world,
                  state.render_ints, state.render_floats, **kw)


def rng(seed: int, pixel: int, sample: int, ndims: int) -> np.ndarray:
    out = np.zeros(ndims, np.float32)
    lib().orc_rng(seed, pixel, sample, ndims, _p(out, ctypes.c_float))
    return out


def disk(u: np.ndarray) -> np.ndarray:
    u = _f32(u).reshape(-1, 2)
    xy = np.zeros_like(u)
    lib().orc_disk(u.shape[0], _p(u, ctypes.c_float), _p(xy, ctypes.c_float))
    return xy


def bsdf_eval(mat12, n, wo, wi):
    m, n, wo, wi = _f32(mat12), _f32(n), _f32(wo), _f32(wi)
    f3, pdf = np.zeros(3, np.float32), np.zeros(1, np.float32)
    lib().orc_bsdf_eval(_p(m, ctypes.c_float), _p(n, ctypes.c_float), _p(wo, ctypes.c_float),
                        _p(wi, ctypes.c_float), _p(f3, ctypes.c_float), _p(pdf, ctypes.c_float))
    return f3, float(pdf[0])


def bsdf_sample(mat12, n, wo, u):
    """sample_bsdf at one shading point for each row (ul, u1, u2) of u:
    (wi [k,3], f [k,3], pdf [k], ok [k] bool)."""
    m, n, wo, u = _f32(mat12), _f32(n), _f32(wo), _f32(u).reshape(-1, 3)
    k = u.shape[0]
    wi, f = np.zeros((k, 3), np.float32), np.zeros((k, 3), np.float32)
    pdf, ok = np.zeros(k, np.float32), np.zeros(k, np.int32)
    lib().orc_bsdf_sample(_p(m, ctypes.c_float), _p(n, ctypes.c_float), _p(wo, ctypes.c_float), k,
                          _p(u, ctypes.c_float), _p(wi, ctypes.c_float), _p(f, ctypes.c_float),
                          _p(pdf, ctypes.c_float), _p(ok, ctypes.c_int32))
    return wi, f, pdf, ok.astype(bool)


def bsdf_sample_lobes(mat12, n, wo, u):
    """bsdf_sample with the lobe: ok 0 (path ends), 1 diffuse, 2 glossy (rr_debug_bsdf_sample)."""
    m, n, wo, u = _f32(mat12), _f32(n), _f32(wo), _f32(u).reshape(-1, 3)
    k = u.shape[0]
    wi, f = np.zeros((k, 3), np.float32), np.zeros((k, 3), np.float32)
    pdf, ok = np.zeros(k, np.float32), np.zeros(k, np.int32)
    lib().orc_bsdf_sample(_p(m, ctypes.c_float), _p(n, ctypes.c_float), _p(wo, ctypes.c_float), k,
                          _p(u, ctypes.c_float), _p(wi, ctypes.c_float), _p(f, ctypes.c_float),
                          _p(pdf, ctypes.c_float), _p(ok, ctypes.c_int32))
    return wi, f, pdf, ok


def bsdf_eval_n(mat12, n, wo, wi):
    """eval_bsdf at one shading point for each row of wi: (f [k,3], pdf [k])."""
    m, n, wo, wi = _f32(mat12), _f32(n), _f32(wo), _f32(wi).reshape(-1, 3)
    k = wi.shape[0]
    f, pdf = np.zeros((k, 3), np.float32), np.zeros(k, np.float32)
    lib().orc_bsdf_eval_n(_p(m, ctypes.c_float), _p(n, ctypes.c_float), _p(wo, ctypes.c_float), k,
                          _p(wi, ctypes.c_float), _p(f, ctypes.c_float), _p(pdf, ctypes.c_float))
    return f, pdf


def filter_table(width: float) -> np.ndarray:
    t = np.zeros(1024, np.float32)
    lib().orc_filter_table(width, _p(t, ctypes.c_float))
    return t


def srgb_lut() -> np.ndarray:
    t = np.zeros(4097, np.float32)
    lib().orc_srgb_lut(_p(t, ctypes.c_float))
    return t


_filmic_keep = None


def set_filmic(luts):
    """LUTs of the Filmic view (render_ints[5] == 2) for the oracle's renders:
    luts = host_oracle.load_filmic_luts(dir) (cube (n,n,n,3), lut1 (n1, comps),
    lo1, hi1), or None to clear."""
    global _filmic_keep
    if luts is None:
        _filmic_keep = None
        lib().orc_set_filmic(None, 0, None, 0, 1, 0.0, 1.0)
        return
    cube = _f32(luts["cube"])
    lut1 = _f32(luts["lut1"])
    _filmic_keep = (cube, lut1)
    lib().orc_set_filmic(_p(cube, ctypes.c_float), int(cube.shape[0]), _p(lut1, ctypes.c_float),
                         int(lut1.shape[0]), int(lut1.shape[1]), float(luts["lo1"]), float(luts["hi1"]))


def filmic(rgb: np.ndarray) -> np.ndarray:
    """Filmic 8-bit code values of linear RGB triples (set_filmic first)."""
    rgb = _f32(rgb).reshape(-1, 3)
    out = np.zeros((rgb.shape[0], 3), np.uint8)
    lib().orc_filmic(rgb.shape[0], _p(rgb, ctypes.c_float), _p(out, ctypes.c_uint8))
    return out


def material_lut(mat12) -> np.ndarray:
    """The material's table (Fresnel blend | lobe pick probability, 260 floats)."""
    m = _f32(mat12)
    out = np.zeros(260, np.float32)
    lib().orc_material_lut(_p(m, ctypes.c_float), _p(out, ctypes.c_float))
    return out


def last_build_seconds() -> float:
    """Wall seconds the last render() spent building its hierarchy."""
    L = lib()
    L.orc_last_build_seconds.restype = ctypes.c_double
    return float(L.orc_last_build_seconds())


def camera_rays(state, pixels, samples) -> np.ndarray:
    """Camera rays (n, 8: o, tmin, d, tmax) of the (pixel, sample) pairs of a
    FrameState's frame, as the oracle's radiance() starts them."""
    pix = np.ascontiguousarray(pixels, dtype=np.int32)
    smp = np.ascontiguousarray(samples, dtype=np.int32)
    cam, ri, rf = _f32(state.camera), np.ascontiguousarray(state.render_ints, np.int32), _f32(state.render_floats)
    out = np.zeros((len(pix), 8), np.float32)
    lib().orc_camera_rays(_p(cam, ctypes.c_float), _p(ri, ctypes.c_int32), _p(rf, ctypes.c_float), len(pix),
                          _p(pix, ctypes.c_int32), _p(smp, ctypes.c_int32), _p(out, ctypes.c_float))
    return out


def stack_drops(reset: bool = False) -> int:
    """Traversal-stack pushes the oracle dropped for want of room (ORC_MAXDEPTH)
    since the last reset: each a missed subtree (rr_frame_stats.stack_drops on
    the GPU)."""
    L = lib()
    L.orc_stack_drops.restype = ctypes.c_longlong
    n = int(L.orc_stack_drops())
    if reset:
        L.orc_reset_stack_drops()
    return n


def ray_counts():
    """Ray statistics of the last render (test/debug): (continuations at bounce 0,
    shadow rays at bounce 0, continuations later, shadow rays later) and the
    first (pixel, sample) pairs whose path continued past bounce 1."""
    out = np.zeros(4, np.int64)
    late = np.zeros(32, np.int32)
    n = ctypes.c_int(0)
    lib().orc_ray_counts(_p(out, ctypes.c_longlong), _p(late, ctypes.c_int32), ctypes.byref(n))
    return tuple(int(x) for x in out), [tuple(late[2 * k:2 * k + 2]) for k in range(n.value)]
