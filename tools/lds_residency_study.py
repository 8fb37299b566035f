#!/usr/bin/env python3
"""k_tiles against the split path on LDS-resident scenes of growing size (the
residency cap of wavefront.hip scene_in_lds / the k_tiles LDS footprint).

Each scene is the 04vs stand-in with its cube replaced by a dense soup of
n triangles (icosahedral blobs + shards, tests/soups.py style, seeded): k_tiles
stages nodes, triangles, normals, shading frames and per-triangle camera data
in LDS, about 400 B per triangle, so its blocks per CU fall as n grows. Per n:
the best of three solo renders of frame 5 at 1920x1080 x 128 spp through
k_tiles (the default) and through the split kernels (RR_FLAG_WAVEFRONT), the
k_tiles LDS bytes per block and the blocks per CU they allow.

  python tools/lds_residency_study.py [n ...]      (GPU box)
"""
import importlib
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"


def dense_soup(n: int, seed: int = 1) -> np.ndarray:
    import soups
    rng = np.random.default_rng(seed)
    tris = []
    k = 0
    while len(tris) + 20 <= n - 2:
        c = np.array([-0.9 + 0.6 * (k % 4), -0.6 + 0.6 * (k // 4 % 3), 0.0])
        v = (soups._ico_vertices() * rng.uniform(0.2, 0.3, 12)[:, None]) @ soups._rotation(rng).T + c
        tris.extend(v[soups._ICO_F])
        k += 1
    while len(tris) < n - 2:
        c = rng.uniform(-0.8, 0.8, 3)
        tris.append(c + rng.normal(0.0, 0.15, (3, 3)))
    z = -1.3
    tris.append([[-2.5, -2.5, z], [2.5, -2.5, z], [2.5, 2.5, z]])
    tris.append([[-2.5, -2.5, z], [2.5, 2.5, z], [-2.5, 2.5, z]])
    return np.array(tris[:n], np.float32)


def lds_bytes(n: int, n_mats: int = 2, n_lights: int = 1) -> int:
    """k_tiles' LDS per block (wavefront.hip TileGrid: scene_lds_bytes + camera data + the static stack)."""
    f4 = 4 * max(n - 1, 1) + 3 * n + (3 + 4 + 65) * n_mats + 3 * n_lights + 256 + 5 * n + 13 * n
    return 16 * f4 + 12 * 256 * 4


def main():
    ns = [int(x) for x in sys.argv[1:]] or [12, 30, 50, 70, 90]
    rr = importlib.import_module(PKG)
    base = os.path.join(ROOT, "scenes", "04_very-simple-standin.rrscene")
    d = tempfile.mkdtemp()
    out = {}
    with rr.RenderContext(0) as ctx:
        for n in ns:
            scene = json.load(open(base))
            tris = dense_soup(n)
            mesh = scene["meshes"][0]
            mesh["vertices"] = [float(x) for x in tris.reshape(-1)]
            mesh["triangles"] = list(range(3 * len(tris)))
            mesh["material_indices"] = [0] * len(tris)
            mesh["smooth"] = [0] * len(tris)
            path = os.path.join(d, f"soup{n}.rrscene")
            json.dump(scene, open(path, "w"))
            s = ctx.load_scene(path)
            row = {"lds_bytes_per_block": lds_bytes(n), "blocks_per_cu": 160 * 1024 // lds_bytes(n)}
            for name, flags in (("tiles", 0), ("split", rr.native.RR_FLAG_WAVEFRONT)):
                p = rr.default_params(flags=flags | rr.native.RR_FLAG_PROFILE_KERNELS)
                ctx.render_to_memory(s, 5, p, film=False, rgba=True)
                best = min(sum(ctx.render_to_memory(s, 5, p, film=False, rgba=True)[2].kernel_ms) for _ in range(3))
                row[name + "_ms"] = round(best, 3)
            s.close()
            out[n] = row
            print(n, row, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
