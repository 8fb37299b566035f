"""Host logic of the worker side of the render step, no GPU: the mirror of the
reference's frame queue (worker/src/rendering/queue.rs:42-229) with two frames
in flight, and the trace records of pipelined frames under the reference's
own per-worker accounting (shared/src/results/performance.rs:47-143).

The runner / context below are stand-ins that render nothing: they only let
the tests decide when a frame's device work "finishes"."""
import os
import threading
import time
import types

import pytest

from conftest import ROOT
from oracle import host_oracle as HO


def _job(rr, tmp_path):
    job = rr.BlenderJob.load_from_file(os.path.join(ROOT, "jobs", "04_very-simple_demo_10f-1w.toml"))
    return rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": str(tmp_path / "out")})


class GatedRunner:
    """submit_frame returns at once; complete_frame blocks until the test opens
    the frame's gate (the device work of that frame is 'done')."""

    def __init__(self, fail=()):
        self.gates = {}
        self.submitted = []
        self.completed = []
        self.fail = set(fail)
        self.lock = threading.Lock()

    def gate(self, f):
        with self.lock:
            return self.gates.setdefault(f, threading.Event())

    def submit_frame(self, job, f):
        self.submitted.append(f)
        return f

    def complete_frame(self, f):
        assert self.gate(f).wait(10), f"frame {f} never released"
        self.completed.append(f)
        if f in self.fail:
            raise RuntimeError(f"render of frame {f} failed")
        return None, None


def _wait(pred, timeout=5.0):
    t0 = time.monotonic()
    while not pred():
        if time.monotonic() - t0 > timeout:
            return False
        time.sleep(0.002)
    return True


def test_steal_of_in_flight_and_queued_frames(rr, tmp_path):
    job = _job(rr, tmp_path)
    runner = GatedRunner()
    finished = []
    q = rr.WorkerAutomaticQueue(runner, on_finished=lambda name, f: finished.append(f))
    R = rr.FrameQueueRemoveResult
    try:
        for f in (1, 2, 3, 4):
            q.queue_frame(job, f)
        # frame 1 renders, frame 2 is submitted behind it: both RENDERING
        assert _wait(lambda: runner.submitted == [1, 2])
        st = dict(q.states())
        assert st[1] is st[2] is rr.WorkerFrameState.RENDERING
        assert st[3] is st[4] is rr.WorkerFrameState.QUEUED
        assert q.unqueue_frame(job.job_name, 1)[0] is R.ALREADY_RENDERING
        assert q.unqueue_frame(job.job_name, 2)[0] is R.ALREADY_RENDERING  # the in-flight next frame
        assert q.unqueue_frame(job.job_name, 3)[0] is R.REMOVED_FROM_QUEUE  # a queued frame is stolen
        assert q.unqueue_frame(job.job_name, 3) == (R.ERRORED, "Can't find such queued frame.")
        assert q.unqueue_frame("another job", 4)[0] is R.ERRORED
        runner.gate(1).set()
        assert _wait(lambda: finished == [1])
        assert _wait(lambda: runner.submitted == [1, 2, 4])  # the stolen frame 3 is never rendered
        assert q.unqueue_frame(job.job_name, 4)[0] is R.ALREADY_RENDERING
        runner.gate(2).set()
        runner.gate(4).set()
        assert q.wait_idle(5)
        assert finished == [1, 2, 4] and runner.completed == [1, 2, 4]
        assert q.states() == []
    finally:
        q.cancel()
        for g in runner.gates.values():
            g.set()
        q.join(5)


def test_wakeup_without_poll(rr, tmp_path):
    """queue_frame wakes the loop at once (the reference sleeps 100 ms per loop
    iteration, queue.rs:81)."""
    job = _job(rr, tmp_path)
    runner = GatedRunner()
    q = rr.WorkerAutomaticQueue(runner)
    try:
        time.sleep(0.05)  # the loop is waiting
        t0 = time.monotonic()
        q.queue_frame(job, 7)
        assert _wait(lambda: runner.submitted == [7], 2.0)
        assert time.monotonic() - t0 < 0.05
        runner.gate(7).set()
        assert q.wait_idle(5)
    finally:
        q.cancel()
        q.join(5)


def test_serial_depth_and_failed_frame(rr, tmp_path):
    """frames_in_flight=1 is the reference's serial loop; a failed render is
    logged and dropped, never reported as finished (queue.rs:169-174)."""
    job = _job(rr, tmp_path)
    runner = GatedRunner(fail={2})
    finished = []
    q = rr.WorkerAutomaticQueue(runner, on_finished=lambda n, f: finished.append(f), frames_in_flight=1)
    try:
        for f in (1, 2, 3):
            q.queue_frame(job, f)
        assert _wait(lambda: runner.submitted == [1])
        time.sleep(0.05)
        assert runner.submitted == [1]  # no second frame in flight
        for f in (1, 2, 3):
            runner.gate(f).set()
        assert q.wait_idle(5)
        assert finished == [1, 3]
        assert [f for f, _ in q.errors] == [2]
    finally:
        q.cancel()
        q.join(5)
    with pytest.raises(ValueError):
        rr.WorkerAutomaticQueue(runner, frames_in_flight=rr.native.RR_MAX_FRAMES_IN_FLIGHT + 1)


def test_cancel_stops_taking_frames(rr, tmp_path):
    job = _job(rr, tmp_path)
    runner = GatedRunner()
    q = rr.WorkerAutomaticQueue(runner)
    q.queue_frame(job, 1)
    assert _wait(lambda: runner.submitted == [1])
    q.cancel()
    q.queue_frame(job, 2)
    runner.gate(1).set()
    q.join(5)
    assert not q._thread.is_alive()
    assert runner.submitted == [1]


class FakeCtx:
    """Stand-in for RenderContext with the timing behaviour of two frames in
    flight: a frame's device work starts when it is submitted or when the
    previous frame's ends, and lasts `device_s`; complete() returns the five
    timestamps the C ABI reports (rr_frame_timing) and sleeps for the write."""

    def __init__(self, device_s=0.02, write_s=0.01):
        self.device_s, self.write_s = device_s, write_s
        self.busy_until = 0.0
        self.jobs = {}
        self.next = 1

    def load_scene(self, path):
        return types.SimpleNamespace(close=lambda: None)

    def submit_frame(self, scene, f, params, out, fmt, q):
        now = time.time()
        start = max(now, self.busy_until)
        self.busy_until = start + self.device_s
        t = self.next
        self.next += 1
        self.jobs[t] = (now, start, self.busy_until)
        return t

    def complete_frame(self, t):
        sub, start, end = self.jobs.pop(t)
        while time.time() < end:
            time.sleep(0.001)
        time.sleep(self.write_s)
        timing = types.SimpleNamespace(loaded_at=sub, started_rendering_at=start, finished_rendering_at=end,
                                       file_saving_started_at=end,
                                       file_saving_finished_at=time.time())
        return timing, types.SimpleNamespace(spp=1)

    def render_frame(self, scene, f, params, out, fmt, q):
        return self.complete_frame(self.submit_frame(scene, f, params, out, fmt, q))

    def close(self):
        pass


def test_pipelined_trace_passes_reference_accounting(rr, tmp_path):
    """Frames submitted while the previous one is in flight still yield
    consecutive, non-overlapping FrameRenderTime records: the reference's
    WorkerPerformance (every duration .to_std(), i.e. >= 0) accepts the trace."""
    job = _job(rr, tmp_path)
    tracer = rr.WorkerTraceBuilder()
    runner = rr.BackendRunner(ROOT, tracer=tracer, ctx=FakeCtx())
    tracer.set_job_start_time(time.time())
    frts = runner.render_frames(job, list(range(1, 9)))
    runner.render_frame(job, 9)  # a serial frame after the pipelined ones
    tracer.set_job_finish_time(time.time())
    trace = tracer.build().to_dict()
    perf = HO.worker_performance(trace)  # raises on any negative duration
    assert perf["total_frames_rendered"] == 9
    recs = [f["details"] for f in trace["frame_render_traces"]]
    for a, b in zip(recs, recs[1:]):
        assert b["started_process_at"] >= a["exited_process_at"]
    for r in recs:
        vals = [r[k] for k in rr.traces.FRAME_FIELDS]
        assert vals == sorted(vals)
    assert len(frts) == 8
    # without the clamp the raw submit times overlap (the bug the clamp fixes)
    tm = types.SimpleNamespace(loaded_at=recs[1]["finished_loading_at"],
                               started_rendering_at=recs[1]["started_rendering_at"],
                               finished_rendering_at=recs[1]["finished_rendering_at"],
                               file_saving_started_at=recs[1]["file_saving_started_at"],
                               file_saving_finished_at=recs[1]["file_saving_finished_at"])
    raw = rr.FrameRenderTime.from_timing(recs[1]["started_process_at"] - 1.0, tm, recs[1]["exited_process_at"],
                                         not_before=recs[0]["exited_process_at"])
    assert raw.started_process_at == recs[0]["exited_process_at"]


def test_worker_performance_rejects_overlap():
    fr = {k: 1.0 for k in ("started_process_at", "finished_loading_at", "started_rendering_at",
                           "finished_rendering_at", "file_saving_started_at", "file_saving_finished_at",
                           "exited_process_at")}
    f2 = dict(fr, started_process_at=0.5, finished_loading_at=1.0)
    f3 = dict(fr)
    trace = {"job_start_time": 0.0, "job_finish_time": 2.0,
             "frame_render_traces": [{"details": fr}, {"details": f2}, {"details": f3}]}
    with pytest.raises(ValueError, match="Invalid idle duration"):
        HO.worker_performance(trace)
