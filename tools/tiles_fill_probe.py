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

import numpy as np

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
        if hasattr(ctx, "tile_costs"):
            # the units of the last frame (one of the solo renders): per tile, ticks of 10 ns summed
            # over its slices; the box tiles in the hand-out order that launch used
            costs, order = ctx.tile_costs()
            n = ((st.width + 7) // 8) * ((st.height + 7) // 8)
            c = costs[:n].astype(np.float64) * 1e-5  # ms
            box = int(np.count_nonzero(c))
            unit = c[c > 0] / max(st.tile_slices, 1)
            o = order[:box]
            pos = {int(t): i for i, t in enumerate(o)}
            heavy = np.argsort(-c)[:20]
            out.update({"box_tiles": box, "unit_ms_mean": round(float(unit.mean()), 4) if box else 0,
                        "unit_ms_p99": round(float(np.percentile(unit, 99)), 4) if box else 0,
                        "unit_ms_max": round(float(unit.max()), 4) if box else 0,
                        "sum_unit_ms_over_waves": round(float(c.sum()) / 4096.0, 4),
                        "heaviest_20_order_positions": [pos.get(int(t), -1) for t in heavy],
                        "cost_decile_ms_by_order": [round(float(c[o[i * box // 10:(i + 1) * box // 10]].mean()), 4)
                                                    for i in range(10)] if box >= 10 else []})
        print(json.dumps(out), flush=True)
        s.close()


if __name__ == "__main__":
    main()
