#!/usr/bin/env python3
"""Traversal diagnostics of one frame of a scene (GPU box): LBVH depth
histogram (from the device build), node visits / triangle tests per ray for
each kernel class (RR_FLAG_COUNT_TRAVERSAL), ray counts and per-kernel times.
  python tools/diag_traversal.py scenes/02_physics-standin.rrscene 90 [spp]"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")


def depths(children: np.ndarray) -> np.ndarray:
    n_in = children.shape[0]
    d = np.zeros(n_in, np.int32)
    leaf_d = []
    stack = [(0, 0)]
    while stack:
        v, k = stack.pop()
        d[v] = k
        for c in children[v]:
            if c >= 0:
                stack.append((int(c), k + 1))
            else:
                leaf_d.append(k + 1)
    return np.array(leaf_d)


def main():
    path, frame = sys.argv[1], int(sys.argv[2])
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    with rr.RenderContext(0) as ctx:
        s = ctx.load_scene(path)
        _, _, children, _ = ctx.bvh(s, frame)
        ld = depths(children)
        out = {"scene": os.path.basename(path), "frame": frame, "triangles": int(children.shape[0] + 1),
               "leaf_depth": {"mean": float(ld.mean()), "max": int(ld.max()),
                              "p99": float(np.percentile(ld, 99)), "frac_gt_16": float((ld > 16).mean()),
                              "frac_gt_32": float((ld > 32).mean())}}
        p = rr.default_params(spp=spp, flags=rr.native.RR_FLAG_PROFILE_KERNELS)
        ctx.render_to_memory(s, frame, p, film=False, rgba=True)
        _, _, st = ctx.render_to_memory(s, frame, p, film=False, rgba=True)
        names = rr.native.KERNEL_CLASSES
        out["kernel_ms"] = {names[k]: round(st.kernel_ms[k], 3) for k in range(len(names))}
        out["launches"] = {names[k]: int(st.kernel_launches[k]) for k in range(len(names))}
        p = rr.default_params(spp=spp, flags=rr.native.RR_FLAG_COUNT_TRAVERSAL)
        _, _, c = ctx.render_to_memory(s, frame, p, film=False, rgba=True)
        rays = {"primary": c.camera_rays, "extend": c.extension_rays, "shadow": c.shadow_rays}
        out["rays"] = {k: int(v) for k, v in rays.items()}
        out["nodes_per_ray"] = {k: round(c.trav_nodes[i] / max(rays[k], 1), 2) for i, k in enumerate(rays)}
        out["tris_per_ray"] = {k: round(c.trav_tris[i] / max(rays[k], 1), 2) for i, k in enumerate(rays)}
        out["grays_per_s"] = {k: round(rays[k] / max(st.kernel_ms[names.index(k)], 1e-9) / 1e6, 3) for k in rays}
        s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
