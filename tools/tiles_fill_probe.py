#!/usr/bin/env python3
"""k_tiles wave fill of a lone frame (GPU box): renders one frame with
RR_FLAG_COUNT_TRAVERSAL and prints the counting launch's wave fill, the spread
of its wave starts and ends over the launch (rr_frame_stats
kernel_wave_fill / kernel_entry_spread / kernel_exit_spread) and the best of
three solo kernel times. The library comes from RR_LIB_PATH when set (A/B).

  python tools/tiles_fill_probe.py [scene] [frame] [spp]
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "04_very-simple-standin.rrscene")
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rr = importlib.import_module(PKG)
    with rr.RenderContext(0) as ctx:
        s = ctx.load_scene(scene)
        kw = {"spp": spp} if spp else {}
        pc = rr.default_params(flags=rr.native.RR_FLAG_COUNT_TRAVERSAL, **kw)
        pt = rr.default_params(flags=rr.native.RR_FLAG_PROFILE_KERNELS, **kw)
        ctx.render_to_memory(s, frame, pt, film=False, rgba=True)
        st = ctx.render_to_memory(s, frame, pc, film=False, rgba=True)[2]
        best = min(sum(ctx.render_to_memory(s, frame, pt, film=False, rgba=True)[2].kernel_ms) for _ in range(3))
        out = {"lib": os.environ.get("RR_LIB_PATH", "in-tree"), "wave_fill": round(st.kernel_wave_fill, 3),
               "entry_spread": round(st.kernel_entry_spread, 3), "exit_spread": round(st.kernel_exit_spread, 3),
               "tile_slices": st.tile_slices, "solo_kernel_ms": round(best, 3)}
        print(json.dumps(out), flush=True)
        s.close()


if __name__ == "__main__":
    main()
