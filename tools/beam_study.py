#!/usr/bin/env python3
"""Work of the bounce-0 shadow-ray beam packets (the device walk
packet_shadow_beam of commit 76f0210, measured slower and removed) against
per-lane any-hit walks, on the CPU (research):
the oracle built with ORC_WALK_STUDY runs the device's beam walk over packets
of one pixel's shadow rays and checks that every ray's occlusion equals the
per-lane walk's. Rays: `spp` camera rays per sampled pixel, their hits, and a
shadow ray from each toward a light chosen uniformly per sample (a random
point of a disk light's disk, a sun's direction), as shade() casts them.
Packets: one pixel's rays together ("mixed"), or split by light ("by light").
  python tools/beam_study.py [02|03|c5] [frame] [n_pixels] [spp]"""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import oracle as O  # noqa: E402
import walk_study as WS  # noqa: E402

PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"
SCENES = {"02": "02_physics-standin", "03": "03_physics-2-standin", "c5": "c5_synthetic-10m"}


def shadow_rays(tris, st, npx, spp, rng):
    W, H = int(st.render_ints[0]), int(st.render_ints[1])
    pix = np.repeat(rng.integers(0, W * H, npx).astype(np.int32), spp)
    smp = np.tile(np.arange(spp, dtype=np.int32), npx)
    cam = O.camera_rays(st, pix, smp)
    h, p, _ = O.trace(tris, cam, width=4)
    hit = p >= 0
    P = cam[:, 0:3].astype(np.float64) + h[:, 0:1].astype(np.float64) * cam[:, 4:7].astype(np.float64)
    t = tris[np.maximum(p, 0)].astype(np.float64)
    n = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
    n *= -np.sign(np.einsum("ij,ij->i", n, cam[:, 4:7]))[:, None]
    Po = P + 1e-4 * n
    lights = np.asarray(st.lights, np.float32).reshape(-1, 12)
    li = rng.integers(0, len(lights), len(Po))
    d = np.zeros_like(Po)
    dist = np.zeros(len(Po))
    for k, lt in enumerate(lights):
        sel = li == k
        if lt[0] == 0.0:  # point / disk light: a random point of the disk facing the point
            lp = lt[1:4].astype(np.float64)
            wl = lp - Po[sel]
            wl /= np.linalg.norm(wl, axis=1, keepdims=True)
            a = np.where(np.abs(wl[:, :1]) > 0.9, [[0.0, 1.0, 0.0]], [[1.0, 0.0, 0.0]])
            b1 = np.cross(wl, a)
            b1 /= np.linalg.norm(b1, axis=1, keepdims=True)
            b2 = np.cross(wl, b1)
            r = lt[7] * np.sqrt(rng.random(sel.sum()))[:, None]
            ph = 2 * np.pi * rng.random(sel.sum())[:, None]
            sp = lp + r * (np.cos(ph) * b1 + np.sin(ph) * b2)
            v = sp - Po[sel]
            dist[sel] = np.linalg.norm(v, axis=1)
            d[sel] = v / dist[sel][:, None]
        else:  # sun
            d[sel] = -lt[4:7]
            dist[sel] = 3.0e38
    rays = np.concatenate([Po, np.zeros((len(Po), 1)), d, dist[:, None]], axis=1).astype(np.float32)
    return rays, hit, li


def fov_x(st):
    """Horizontal field of view of the frame's camera (radians): from the
    camera block's half width at unit distance when the binding exposes it."""
    import math
    cam = np.asarray(st.camera, np.float64)
    return 2.0 * math.atan(float(cam[12])) if cam.size > 12 else math.radians(39.6)


def run(L, tris, rays, groups):
    """The beam study over packets = the index groups (one hierarchy build)."""
    idx = np.concatenate(groups)
    starts = np.concatenate([[0], np.cumsum([len(g) for g in groups])]).astype(np.int32)
    r = np.ascontiguousarray(rays[idx])
    out = np.zeros(7, np.int64)
    L.orc_study_beam(tris.shape[0], tris.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(groups),
                     starts.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                     r.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
    return out


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else "02"
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 90
    npx = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    spp = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    WS.build_study_lib()
    O.LIB = WS.STUDY_LIB
    import collapse_study as CS
    L = O.lib()
    L.orc_set_walk_counting(1)
    rr = importlib.import_module(PKG)
    path = os.path.join(ROOT, "scenes", SCENES[key] + ".rrscene")
    s = rr.Scene(path)
    st = s.frame_constants(frame)
    tris = np.ascontiguousarray(CS.world_tris(path, s, frame).astype(np.float32))
    s.close()
    rng = np.random.default_rng(1)
    rays, hit, li = shadow_rays(tris, st, npx, spp, rng)
    keep = hit.reshape(npx, spp)
    print(f"{key} frame {frame}: {len(tris)} triangles, {npx} pixels x {spp} samples")
    # mixed: one pixel's rays of camera hits in one packet (padding: repeat the pixel's first ray)
    # the device's spread test (beam_coherent of commit 76f0210): origins within 4 pixel footprints
    cam_pos = np.asarray(st.camera, np.float64)[:3]

    def coherent(g, spread=4.0):
        o = rays[g, 0:3].astype(np.float64)
        dc = np.abs(o - cam_pos).max()
        return (o.max(0) - o.min(0)).max() <= spread * 1.7320508 * dc * pix_angle

    W = int(st.render_ints[0])
    pix_angle = 2.0 * np.tan(0.5 * fov_x(st)) / W
    by_light = [g for i in range(npx) for k in range(li.max() + 1)
                for g in [np.flatnonzero(keep[i] & (li[i * spp:(i + 1) * spp] == k)) + i * spp] if len(g)]
    lights = np.asarray(st.lights, np.float32).reshape(-1, 12)
    cases = [("mixed", [np.flatnonzero(keep[i]) + i * spp for i in range(npx)]), ("by light", by_light)]
    for k in range(len(lights)):
        gk = [g for g in by_light if li[g[0]] == k]
        kind = "disk" if lights[k][0] == 0.0 else "sun"
        cases.append((f"{kind}, coherent", [g for g in gk if coherent(g)]))
        cases.append((f"{kind}, not", [g for g in gk if not coherent(g)]))
    for name, groups in cases:
        groups = [g for g in groups if len(g)]
        if not groups:
            continue
        tot = run(L, tris, rays, groups)
        n = max(sum(len(g) for g in groups), 1)
        print(f"  {name:8s}: {tot[0]} packets; beam {tot[1] / tot[0]:.1f} node visits per packet, "
              f"{tot[2] / n:.1f} leaf tests per ray; per-lane {tot[3] / n:.1f} node visits, {tot[4] / n:.1f} "
              f"leaf tests per ray; blocked {tot[6] / n:.3f}; occlusion mismatches {tot[5]}")


if __name__ == "__main__":
    main()
