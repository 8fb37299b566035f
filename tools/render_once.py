#!/usr/bin/env python3
"""Render one frame of a scene a few times through render_to_memory (the
library named by RR_LIB_PATH, else the in-tree build): a short program for
rocprofv3 passes over a single kernel variant.
  python tools/render_once.py [frame] [scene] [repeats]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")

frame = int(sys.argv[1]) if len(sys.argv) > 1 else 1
scene = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "scenes", "04_very-simple-standin.rrscene")
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
with rr.RenderContext(0) as ctx:
    s = ctx.load_scene(scene)
    for _ in range(reps):
        ctx.render_to_memory(s, frame, rr.default_params(), film=False, rgba=True)
    s.close()
