#!/usr/bin/env python3
"""Golden row digests of whole split-path frames at the bench size, for
tests/test_gpu_physics.py test_bench_size_split_frames_match_oracle_fixture:
02 frame 90 and 03 frame 300 at 1920x1080 x 64 spp (the scenes' defaults, what
bench.py --workload 02 / 03 renders).

  on the GPU box:  python tools/make_split_golden.py dump
                   -> gpurun_out/split_state_<scene>_<frame>.npz
  here (CPU):      python tools/make_split_golden.py render [--threads N]
                   -> tests/golden/split_full_frames.json

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


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("dump")
    r = sub.add_parser("render")
    r.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    r.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    {"dump": cmd_dump, "render": cmd_render}[a.cmd](a)


if __name__ == "__main__":
    main()
