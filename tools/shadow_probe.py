#!/usr/bin/env python3
"""Per-class kernel times of split-path frames at growing sizes (GPU box,
research): one line per (scene, size), printed as soon as it is rendered, so a
run under `timeout` shows how far it got.
  python tools/shadow_probe.py SCENE:FRAME:W:H:SPP ..."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")

with rr.RenderContext(0) as ctx:
    for spec in sys.argv[1:]:
        path, frame, w, h, spp = spec.split(":")
        s = ctx.load_scene(os.path.join(ROOT, "scenes", path))
        p = rr.default_params(width=int(w), height=int(h), spp=int(spp), flags=rr.native.RR_FLAG_PROFILE_KERNELS)
        t0 = time.time()
        _, _, st = ctx.render_to_memory(s, int(frame), p, film=False, rgba=True)
        ms = {n: round(st.kernel_ms[k], 3) for k, n in enumerate(rr.native.KERNEL_CLASSES) if st.kernel_ms[k] > 0}
        print(f"{spec}: {time.time() - t0:.2f} s wall, kernels {ms}, shadow rays {st.shadow_rays}", flush=True)
        s.close()
