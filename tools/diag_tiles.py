"""Diagnostic: k_tiles vs oracle mismatches for small frames."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")
from oracle import oracle as O
ctx = rr.RenderContext(0)
s = ctx.load_scene(os.path.join(ROOT, "scenes", "04_very-simple-standin.rrscene"))
for (frame, w, h, spp, flags) in [(45, 7, 130, 3, 0), (45, 7, 130, 3, 4), (45, 7, 130, 1, 0), (45, 16, 130, 3, 0),
                                  (45, 64, 130, 3, 0), (30, 7, 130, 3, 0), (45, 8, 130, 3, 0)]:
    p = rr.default_params(width=w, height=h, spp=spp, flags=flags)
    film, rgba, st = ctx.render_to_memory(s, frame, p)
    of, orgba = O.render_state(ctx.frame_state(s, frame, p))
    bad = np.nonzero(np.any(film != of, axis=-1))
    print(frame, w, h, spp, flags, "mismatched px", len(bad[0]), flush=True)
    for y, x in list(zip(*bad))[:4]:
        print("   ", y, x, film[y, x, :3], of[y, x, :3])
s.close()
ctx.close()
