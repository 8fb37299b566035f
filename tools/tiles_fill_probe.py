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
        solo_log = os.environ.get("RR_PROBE_SOLO_LOG") == "1"  # a library built with RR_TILES_LOG_ALWAYS=1
        prev_costs = None
        if solo_log:  # the unit log of the last solo (non-counting) launch
            st = ctx.render_to_memory(s, frame, pc, film=False, rgba=True)[2]
            ctx.render_to_memory(s, frame, pt, film=False, rgba=True)
            prev_costs = ctx.tile_costs(units=0)[0].copy()  # recorded by the launch 3 frames (one slot) before the last
            best = min(sum(ctx.render_to_memory(s, frame, pt, film=False, rgba=True)[2].kernel_ms) for _ in range(3))
        else:  # the counting launch's
            best = min(sum(ctx.render_to_memory(s, frame, pt, film=False, rgba=True)[2].kernel_ms) for _ in range(3))
            st = ctx.render_to_memory(s, frame, pc, film=False, rgba=True)[2]
        out = {"lib": os.environ.get("RR_LIB_PATH", "in-tree"), "log_of": "solo" if solo_log else "counting",
               "wave_fill": round(st.kernel_wave_fill, 3),
               "entry_spread": round(st.kernel_entry_spread, 3), "exit_spread": round(st.kernel_exit_spread, 3),
               "tile_slices": st.tile_slices, "solo_kernel_ms": round(best, 3)}
        if hasattr(ctx, "tile_costs"):
            costs, order, log = ctx.tile_costs()
            logged = np.nonzero(log[:, 1])[0]  # box units u (hand-out numbers) of the counting launch
            if logged.size:
                st0 = log[logged, 0].astype(np.float64)
                en = log[logged, 1].astype(np.float64)
                t0 = st0.min()
                span = en.max() - t0
                dur = (en - st0) * 1e-5  # ms
                j = logged // max(st.tile_slices, 1)  # position in the hand-out order
                last = np.argsort(-en)[:10]
                dec = np.array_split(np.argsort(j), 10)
                out.update({
                    "units_logged": int(logged.size), "unit_ms_mean": round(float(dur.mean()), 4),
                    "unit_ms_max": round(float(dur.max()), 4),
                    "last_unit_start_frac": round(float((st0.max() - t0) / span), 3),
                    "unit_ms_by_order_decile": [round(float(dur[d].mean()), 4) for d in dec],
                    "start_frac_by_order_decile": [round(float(((st0[d] - t0) / span).mean()), 3) for d in dec],
                    "last10_ending": [{"u": int(logged[i]), "pos_frac": round(float(j[i]) / max(1, int(j.max())), 3),
                                       "start_frac": round(float((st0[i] - t0) / span), 3),
                                       "ms": round(float(dur[i]), 4)} for i in last]})
            if prev_costs is not None:  # does the last launch's hand-out order follow the costs it was built from?
                nzt = np.nonzero(prev_costs[:((st.width + 7) // 8) * ((st.height + 7) // 8)])[0]
                tx = (st.width + 7) // 8
                if nzt.size:
                    xs, ys = nzt % tx, nzt // tx
                    bx0, by0, bw = int(xs.min()), int(ys.min()), int(xs.max() - xs.min() + 1)
                    bh = int(ys.max() - ys.min() + 1)
                    nb = bw * bh
                    o = order[:nb]
                    if sorted(o.tolist()) == list(range(nb)):
                        scr = (by0 + o // bw) * tx + (bx0 + o % bw)
                        pc_ms = prev_costs[scr].astype(np.float64) * 1e-5
                        out["order_check"] = {"box": [bx0, by0, bw, bh],
                                              "prev_cost_ms_by_order_decile": [round(float(v.mean()), 4) for v in
                                                                               np.array_split(pc_ms, 10)],
                                              "cur_cost_ms_by_order_decile": [round(float(v.mean()), 4) for v in
                                                                              np.array_split(costs[scr].astype(np.float64) * 1e-5, 10)]}
                    else:
                        out["order_check"] = {"box_guess_failed": [bx0, by0, bw, bh]}
        print(json.dumps(out), flush=True)
        s.close()


if __name__ == "__main__":
    main()
