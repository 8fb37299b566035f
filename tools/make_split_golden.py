#!/usr/bin/env python3
"""Golden row digests of whole split-path frames at the bench size, for
tests/test_gpu_physics.py test_bench_size_split_frames_match_oracle_fixture:
02 frame 90 and 03 frame 300 at 1920x1080 x 64 spp (the scenes' defaults, what
bench.py --workload 02 / 03 renders).

  on the GPU box:  python tools/make_split_golden.py dump
                   -> gpurun_out/split_state_<scene>_<frame>.npz
  here (CPU):      python tools/make_split_golden.py render [--threads N]
                   -> tests/golden/split_full_frames.json
  here (CPU):      python tools/make_split_golden.py c5 [--threads N]
                   -> tests/golden/split_full_frame_c5.json

C5 (round 6): frame 150 at 3840x2160 x 64 spp, the bench's resolution with a
sixteenth of its samples (the whole 1024-spp frame would take the oracle about
70 minutes of a 16-thread share). Its 10.5M-triangle state is too large to
bring back from the GPU box, so `c5` builds it on the host without a GPU: the
world triangles by the host restatement that
test_device_world_triangles_match_host_restatement pins the device's
k_transform to (the object poses of oracle/host_oracle.py, rounded to float32,
times the object-space vertices in the kernel's operation order), and the
camera, lights, materials and render settings by the library's host-only frame
evaluation (Scene.frame_constants). The GPU test checks that the device's
frame state digests to the fixture's before comparing rows.

The input is the device's own frame state (rr_debug_frame_state: the world
triangles, camera, lights, materials and render settings the kernels consume;
its world triangles are pinned to the host restatement by
test_device_world_triangles_match_host_restatement). The oracle
(oracle/rr_oracle.c, OpenMP over every core of this container) renders every
row of the frame from it, and the fixture keeps a digest of the state arrays
and one digest per row of the 8-bit image and of the film (float32 RGBA).
Oracle output only: nothing of the reference is read or run.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"
FRAMES = [("02_physics-standin.rrscene", 90), ("03_physics-2-standin.rrscene", 300)]
STATE_FIELDS = ("tris", "tri_mat", "camera", "lights", "materials", "world", "render_ints", "render_floats")
FIXTURE = os.path.join(ROOT, "tests", "golden", "split_full_frames.json")
FIXTURE_C5 = os.path.join(ROOT, "tests", "golden", "split_full_frame_c5.json")
C5 = ("c5_synthetic-10m.rrscene", 150, 64)  # scene, frame, spp (3840x2160: the scene's resolution)


def digest(a: np.ndarray) -> str:
    return hashlib.blake2b(np.ascontiguousarray(a).tobytes(), digest_size=8).hexdigest()


def state_digest(st) -> str:
    h = hashlib.blake2b(digest_size=16)
    for f in STATE_FIELDS:
        a = np.ascontiguousarray(st[f] if isinstance(st, dict) else getattr(st, f))
        h.update(f.encode() + str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def row_digests(img: np.ndarray) -> list:
    return [digest(img[y]) for y in range(img.shape[0])]


def key_of(scene: str, frame: int) -> str:
    return f"{scene.split('.')[0]}:{frame}"


def cmd_dump(a):
    import importlib
    rr = importlib.import_module(PKG)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with rr.RenderContext(0) as ctx:
        for scene, frame in FRAMES:
            s = ctx.load_scene(os.path.join(ROOT, "scenes", scene))
            st = ctx.frame_state(s, frame, rr.default_params())
            s.close()
            out = os.path.join(ROOT, "gpurun_out", f"split_state_{scene.split('_')[0]}_{frame}.npz")
            np.savez_compressed(out, **{f: np.asarray(getattr(st, f)) for f in STATE_FIELDS})
            print(f"{out}: {st.tris.shape[0]} triangles, state {state_digest(st)}", flush=True)


def cmd_render(a):
    from oracle import oracle as O
    fx = {"generator": "tools/make_split_golden.py render (oracle/rr_oracle.c on the device's frame state)",
          "frames": {}}
    for scene, frame in FRAMES:
        path = os.path.join(a.dir, f"split_state_{scene.split('_')[0]}_{frame}.npz")
        with np.load(path) as z:  # our own dump (no pickles: allow_pickle stays False)
            st = {f: z[f] for f in STATE_FIELDS}
        t0 = time.time()
        film, rgba = O.render(st["tris"], st["tri_mat"], st["camera"], st["lights"], st["materials"], st["world"],
                              st["render_ints"], st["render_floats"], threads=a.threads)
        dt = time.time() - t0
        ri = st["render_ints"]
        fx["frames"][key_of(scene, frame)] = {
            "width": int(ri[0]), "height": int(ri[1]), "spp": int(ri[2]), "max_bounces": int(ri[3]),
            "triangles": int(st["tris"].shape[0]), "state": state_digest(st),
            "oracle_seconds": round(dt, 1), "oracle_threads": a.threads,
            "rgba8_rows": row_digests(rgba), "film_rows": row_digests(film)}
        print(f"{scene} frame {frame}: {ri[0]}x{ri[1]} x {ri[2]} spp in {dt:.0f} s", flush=True)
    with open(FIXTURE, "w") as fh:
        json.dump(fx, fh, indent=0)
    print(FIXTURE)


def host_world_tris(path: str, scene_obj, frame: int) -> np.ndarray:
    """World triangles by the host restatement (k_transform's order: ((m0 x +
    m1 y) + m2 z) + m3 in float32 with the pose rounded to float32)."""
    from oracle import host_oracle as HO
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


def c5_params(rr):
    return rr.default_params(spp=C5[2])


def c5_host_state(rr) -> dict:
    """C5's frame state built on the host (no GPU): see the module docstring."""
    path = os.path.join(ROOT, "scenes", C5[0])
    s = rr.Scene(path)
    try:
        fc = s.frame_constants(C5[1], c5_params(rr))
        local, _ = s.mesh()
        tris = host_world_tris(path, s, C5[1]).astype(np.float32)
    finally:
        s.close()
    st = {f: np.asarray(getattr(fc, f)) for f in STATE_FIELDS if f != "tris"}
    st["tris"] = np.ascontiguousarray(tris)
    assert st["tri_mat"].shape[0] == tris.shape[0] == local.shape[0]
    return st


def cmd_c5(a):
    import importlib
    from oracle import oracle as O
    rr = importlib.import_module(PKG)
    st = c5_host_state(rr)
    t0 = time.time()
    film, rgba = O.render(st["tris"], st["tri_mat"], st["camera"], st["lights"], st["materials"], st["world"],
                          st["render_ints"], st["render_floats"], threads=a.threads)
    dt = time.time() - t0
    ri = st["render_ints"]
    fx = {"generator": "tools/make_split_golden.py c5 (oracle/rr_oracle.c on the host-built frame state)",
          "frames": {key_of(C5[0], C5[1]): {
              "width": int(ri[0]), "height": int(ri[1]), "spp": int(ri[2]), "max_bounces": int(ri[3]),
              "triangles": int(st["tris"].shape[0]), "state": state_digest(st),
              "oracle_seconds": round(dt, 1), "oracle_threads": a.threads,
              "rgba8_rows": row_digests(rgba), "film_rows": row_digests(film)}}}
    with open(FIXTURE_C5, "w") as fh:
        json.dump(fx, fh, indent=0)
    print(f"{C5[0]} frame {C5[1]}: {ri[0]}x{ri[1]} x {ri[2]} spp in {dt:.0f} s -> {FIXTURE_C5}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("dump")
    r = sub.add_parser("render")
    r.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    r.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    c = sub.add_parser("c5")
    c.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    {"dump": cmd_dump, "render": cmd_render, "c5": cmd_c5}[a.cmd](a)


if __name__ == "__main__":
    main()
