#!/usr/bin/env python3
"""Timeline of the bench's timed region for a k_tiles workload (GPU box,
research): warmup, then N frames through BackendRunner.render_frames as
bench.py times them, and per frame the A11 timestamps (rr_frame_timing, host
clock) relative to the region's start, so the pipeline's fill (before frame
1's device work starts) and drain (after the last frame's device work) can be
read off.
  python tools/pipeline_timeline.py [steps] [warmup] [job] [preheat frames]"""
import importlib
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 5
job_file = sys.argv[3] if len(sys.argv) > 3 else "04_very-simple_demo_10f-1w.toml"
preheat = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # frames rendered before the first warmup

import torch  # noqa: E402  (as bench.py: the HIP runtime librr binds to is torch's)
torch.cuda.set_device(0)
job = rr.BlenderJob.load_from_file(job_file if os.path.isabs(job_file) else os.path.join(ROOT, "jobs", job_file))
out = tempfile.mkdtemp()
job = rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": out})
runner = rr.BackendRunner(ROOT, params=rr.default_params())
n = job.frame_range_to - job.frame_range_from + 1


def frame_of(i):
    return job.frame_range_from + i % n


ev = []  # (kind, ticket, host time, timing)
_sub, _com = runner.ctx.submit_frame, runner.ctx.complete_frame


def submit(*a, **k):
    t = time.time()
    tk = _sub(*a, **k)
    ev.append(("submit", tk, t, time.time(), None))
    return tk


def complete(tk):
    t = time.time()
    r = _com(tk)
    ev.append(("complete", tk, t, time.time(), r[0]))
    return r


runner.ctx.submit_frame, runner.ctx.complete_frame = submit, complete
if preheat:
    runner.render_frames(job, [frame_of(w) for w in range(preheat)])
for rep in range(3):
    runner.render_frames(job, [frame_of(w) for w in range(warmup)])
    runner.ctx.synchronize()
    torch.cuda.synchronize()
    recs = []
    ev.clear()
    t0 = time.time()
    p0 = time.perf_counter()
    runner.render_frames(job, [frame_of(warmup + s) for s in range(steps)],
                         on_frame=lambda f, frt, st: recs.append((f, frt, time.time())))
    runner.ctx.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - p0
    t_end = t0 + el
    ms = lambda t: round((t - t0) * 1e3, 3)  # noqa: E731
    print(f"rep {rep}: {steps} frames in {el * 1e3:.3f} ms ({steps / el:.1f} frames/s)")
    subs = {tk: (a, b) for kind, tk, a, b, _ in ev if kind == "submit"}
    for i, (kind, tk, a, b, tm) in enumerate([e for e in ev if e[0] == "complete"]):
        if i < 4 or i >= steps - 4:
            sa, sb = subs.get(tk, (t0, t0))
            print(f"  ticket {tk}: submit {ms(sa)}..{ms(sb)} render {ms(tm.started_rendering_at)}.."
                  f"{ms(tm.finished_rendering_at)} saved {ms(tm.file_saving_finished_at)} "
                  f"complete called {ms(a)} returned {ms(b)}")
    print(f"  end of region {ms(t_end)}", flush=True)
runner.close()
