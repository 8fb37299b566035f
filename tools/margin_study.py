#!/usr/bin/env python3
"""Node visits and triangle tests per ray of the quantised 6-wide walk with the
box margin of the product (rr_device.h q6_planes, per node) against other
multiples of it, 0 = no margin (CPU, oracle walk, research tool; the rays are
tools/collapse_study.py's: camera rays of the frame, and from their hits a
cosine bounce ray and a shadow ray toward the first light).
  python tools/margin_study.py [02|03|c5] [frame] [n_pixels] [scale ...]"""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import collapse_study as CS  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rays(key, frame, npx):
    rr = importlib.import_module(CS.PKG)
    path = os.path.join(ROOT, "scenes", CS.SCENES[key] + ".rrscene")
    s = rr.Scene(path)
    st = s.frame_constants(frame)
    tris = CS.world_tris(path, s, frame).astype(np.float32)
    s.close()
    W, H = int(st.render_ints[0]), int(st.render_ints[1])
    rng = np.random.default_rng(1)
    pix = rng.integers(0, W * H, npx).astype(np.int32)
    cam = O.camera_rays(st, pix, np.zeros(npx, np.int32))
    h, p, _ = O.trace(tris, cam, width=4)
    hit = p >= 0
    P = cam[hit, 0:3].astype(np.float64) + h[hit, 0:1].astype(np.float64) * cam[hit, 4:7].astype(np.float64)
    t = tris[p[hit]].astype(np.float64)
    n = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    n *= -np.sign(np.einsum("ij,ij->i", n, cam[hit, 4:7]))[:, None]
    Po = P + 1e-4 * n
    u = rng.normal(size=Po.shape)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    d = n + u
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ext = np.concatenate([Po, np.zeros((len(Po), 1)), d, np.full((len(Po), 1), 1e30)], axis=1).astype(np.float32)
    lt = np.asarray(st.lights, np.float32).reshape(-1, 12)[0]
    if lt[0] == 0.0:
        sd = lt[1:4].astype(np.float64) - Po
        dist = np.linalg.norm(sd, axis=1, keepdims=True)
        sd /= dist
    else:
        sd = np.broadcast_to(-lt[4:7].astype(np.float64), Po.shape)
        dist = np.full((len(Po), 1), 3.0e38)
    sh = np.concatenate([Po, np.zeros((len(Po), 1)), sd, dist], axis=1).astype(np.float32)
    return tris, {"camera": cam, "bounce": ext, "shadow": sh}


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else "02"
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 90
    npx = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    scales = [float(x) for x in sys.argv[4:]] or [1.0, 0.25, 0.0]
    tris, sets = rays(key, frame, npx)
    L = O.lib()
    L.orc_set_margin_scale.argtypes = [ctypes.c_float]
    L.orc_set_walk_counting(1)
    out = np.zeros(6, np.int64)
    ptr = out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong))
    print(f"{key} frame {frame}: {len(tris)} triangles")
    for name, r in sets.items():
        for sc in scales:
            L.orc_set_margin_scale(sc)
            L.orc_walk_counts(ptr, 1)
            O.trace(tris, r, width=4)
            L.orc_walk_counts(ptr, 1)
            print(f"  {name:7s} margin x{sc:<5g}: {out[0] / len(r):7.2f} node visits, {out[1] / len(r):6.2f} triangle tests per ray")
    L.orc_set_margin_scale(1.0)
    L.orc_set_walk_counting(0)


if __name__ == "__main__":
    main()
