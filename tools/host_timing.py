#!/usr/bin/env python3
"""Host-side cost of the pipelined worker loop on the GPU box: per frame, the
time spent inside rr_frame_submit and rr_frame_complete (split into waiting
for the device and encode + write, stats.encode_ms), against the device time
of the frame. Tells whether frames/s is bound by the GPU or by the host.
  python tools/host_timing.py [scene] [frames]"""
import importlib
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")


def main():
    scene_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "04_very-simple-standin.rrscene")
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    out = tempfile.mkdtemp(prefix="rr_host_timing_")
    prof = os.environ.get("RR_HOST_TIMING_PROFILE", "0") == "1"
    params = rr.default_params(flags=rr.native.RR_FLAG_PROFILE_KERNELS if prof else 0)
    depth = rr.native.RR_MAX_FRAMES_IN_FLIGHT
    rows = []
    with rr.RenderContext(0) as ctx:
        s = ctx.load_scene(scene_path)
        for f in (1, 2):  # warm-up
            t = ctx.submit_frame(s, f, params, os.path.join(out, f"w{f}"), "JPEG", 90)
            ctx.complete_frame(t)
        pending = []
        t_start = time.perf_counter()
        for i in range(n):
            f = 1 + i % 10
            t0 = time.perf_counter()
            tk = ctx.submit_frame(s, f, params, os.path.join(out, f"{i:06d}"), "JPEG", 90)
            t_sub = time.perf_counter() - t0
            pending.append((tk, t_sub))
            if len(pending) >= depth:
                tk0, ts0 = pending.pop(0)
                t1 = time.perf_counter()
                _, st = ctx.complete_frame(tk0)
                rows.append((ts0, time.perf_counter() - t1, st.encode_ms * 1e-3, st.trace_ms * 1e-3,
                             sum(st.kernel_ms) * 1e-3, st.anim_ms * 1e-3))
        while pending:
            tk0, ts0 = pending.pop(0)
            t1 = time.perf_counter()
            _, st = ctx.complete_frame(tk0)
            rows.append((ts0, time.perf_counter() - t1, st.encode_ms * 1e-3, st.trace_ms * 1e-3,
                         sum(st.kernel_ms) * 1e-3, st.anim_ms * 1e-3))
        wall = time.perf_counter() - t_start
        s.close()
    k = len(rows)
    avg = [sum(r[j] for r in rows) / k * 1e3 for j in range(6)]
    print(f"frames {k}, wall {wall / k * 1e3:.3f} ms/frame ({k / wall:.1f} frames/s)")
    print(f"{depth} frames in flight, per-kernel events {'on' if prof else 'off'}")
    print(f"submit {avg[0]:.3f} ms | complete {avg[1]:.3f} ms (encode+write {avg[2]:.3f}) | "
          f"device trace {avg[3]:.3f} ms, kernels {avg[4]:.3f} ms | anim {avg[5]:.3f} ms")


if __name__ == "__main__":
    main()
