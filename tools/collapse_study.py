#!/usr/bin/env python3
"""Node visits and triangle tests per ray of the quantised 6-wide walk under
two collapses of the same PLOC BVH2 (CPU, oracle walk, research tool):
  0  the product's greedy opening (largest child box first, bvh.hip qw_set)
  1  a surface-area dynamic programme over the BVH2 (Ylitie et al. 2017)
Rays: camera rays of the frame (O.camera_rays over a pixel subsample), and
from their hits a cosine-distributed bounce ray and a shadow ray toward the
scene's first light, as the path tracer casts them.
  python tools/collapse_study.py [02|03|c5] [frame] [n_pixels]"""
import ctypes
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import host_oracle as HO  # noqa: E402
from oracle import oracle as O  # noqa: E402

PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"
SCENES = {"02": "02_physics-standin", "03": "03_physics-2-standin", "c5": "c5_synthetic-10m"}


def world_tris(path, scene_obj, frame):
    scene = HO.load_scene(path)
    bodies = HO.expand_rigid_bodies(scene)
    n_explicit = len(scene["objects"])
    fps, f0 = scene["render"]["fps"], scene["render"]["frame_start"]
    local, obj = scene_obj.mesh()
    mats = np.zeros((n_explicit + len(bodies), 3, 4), np.float32)
    for i in np.unique(obj):
        M = HO.object_matrix(scene["objects"][i], frame) if i < n_explicit else \
            HO.rigid_matrix(bodies[i - n_explicit], (frame - f0) / fps)
        mats[i] = np.asarray(M, np.float64)[:3, :4].astype(np.float32)
    m = mats[obj]
    x, y, z = local[..., 0:1], local[..., 1:2], local[..., 2:3]
    return ((m[:, None, :, 0] * x + m[:, None, :, 1] * y) + m[:, None, :, 2] * z) + m[:, None, :, 3]


def walk(tris, rays, mode):
    L = O.lib()
    L.orc_set_collapse(mode)
    L.orc_set_walk_counting(1)
    out = np.zeros(6, np.int64)
    L.orc_walk_counts(out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), 1)
    t0 = time.time()
    h, p, occ = O.trace(tris, rays, width=4)
    L.orc_walk_counts(out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), 1)
    L.orc_set_collapse(0)
    L.orc_set_walk_counting(0)
    return h, p, occ, out.copy(), time.time() - t0


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else "02"
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 90
    npx = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    rr = importlib.import_module(PKG)
    path = os.path.join(ROOT, "scenes", SCENES[key] + ".rrscene")
    s = rr.Scene(path)
    st = s.frame_constants(frame)
    tris = world_tris(path, s, frame).astype(np.float32)
    W, H = int(st.render_ints[0]), int(st.render_ints[1])
    rng = np.random.default_rng(1)
    pix = rng.integers(0, W * H, npx).astype(np.int32)
    cam = O.camera_rays(st, pix, np.zeros(npx, np.int32))
    h, p, _, c0, _ = walk(tris, cam, 0)
    hit = p >= 0
    # secondary rays from the camera hits: a cosine bounce and a shadow ray
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
    if lt[0] == 0.0:  # point light: toward its centre
        sd = lt[1:4].astype(np.float64) - Po
        dist = np.linalg.norm(sd, axis=1, keepdims=True)
        sd /= dist
    else:  # sun
        sd = np.broadcast_to(-lt[4:7].astype(np.float64), Po.shape)
        dist = np.full((len(Po), 1), 3.0e38)
    sh = np.concatenate([Po, np.zeros((len(Po), 1)), sd, dist], axis=1).astype(np.float32)
    print(f"{key} frame {frame}: {len(tris)} triangles, {npx} camera rays ({hit.mean():.3f} hit), "
          f"{len(ext)} bounce + shadow rays")
    for name, rays in (("camera", cam), ("bounce", ext), ("shadow", sh)):
        res = {}
        for mode in (0, 1):
            hh, pp, oo, cnt, dt = walk(tris, rays, mode)
            res[mode] = (pp, oo, cnt)
            print(f"  {name:7s} collapse {mode}: {cnt[0] / len(rays):7.2f} node visits, {cnt[1] / len(rays):6.2f} "
                  f"triangle tests per ray; of the visits to nodes below 128/256/512/1024: "
                  f"{', '.join(f'{c / len(rays):.2f}' for c in cnt[2:6])} ({dt:.1f} s)")
        assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1]), "results differ"
    s.close()


if __name__ == "__main__":
    main()
