"""BackendRunner — the per-frame render step behind the reference's interface.

Host-side mirror of BlenderJobRunner (/root/reference/worker/src/rendering/runner/mod.rs):
  * __init__  <- BlenderJobRunner::new (:31-70): validates the base directory;
                 instead of a Blender binary it owns one GPU render context.
  * render_frame(job, frame_index) <- render_frame (:72-203): same path
                 resolution (%BASE%), same existence checks and error messages,
                 output directory creation, output naming, the seven
                 FrameRenderTime timestamps and the trace push — but the frame is
                 rendered in-process through the C ABI (include/rr.h) instead of
                 a `blender` subprocess (:165-174), and the project's exported
                 scene is loaded once and cached (the reference re-reads the
                 .blend per frame).
  * submit_frame / complete_frame <- the same step split in two (rr_frame_submit
                 / rr_frame_complete) so the worker can keep its next queued
                 frame in flight.
WorkerAutomaticQueue mirrors the caller, worker/src/rendering/queue.rs.
The Rust worker's equivalent (spawn_blocking over the same C ABI) is in
INTEGRATION.md; these Python classes are what the tests and bench.py drive.
"""
from __future__ import annotations

import enum
import os
import threading
import time
from collections import deque
from dataclasses import dataclass
from pathlib import Path

from .jobs import BlenderJob, JobError, parse_with_base_directory_prefix, scene_path_for_project
from .naming import EXTENSIONS, output_path_without_extension
from .native import RR_MAX_FRAMES_IN_FLIGHT, RenderContext, RenderParams, Scene
from .traces import FrameRenderTime, WorkerTraceBuilder


class RenderError(RuntimeError):
    pass


class BackendRunner:
    def __init__(self, base_directory_path: str | os.PathLike, tracer: WorkerTraceBuilder | None = None,
                 device: int = 0, params: RenderParams | None = None, ctx=None):
        """ctx: a RenderContext on `device` is created here; tests of the host
        logic alone pass a stand-in with the same methods (no rendering)."""
        base = Path(base_directory_path)
        if not base.is_dir():
            raise RenderError("Provided base directory path is not a directory.")
        self.base_directory_path = base
        self.tracer = tracer if tracer is not None else WorkerTraceBuilder()
        self.params = params
        self.ctx = ctx if ctx is not None else RenderContext(device)
        self._scenes: dict[str, Scene] = {}
        self._lock = threading.Lock()  # one caller at a time per context (queue.rs:79-118)
        self.last_stats = None
        self._last_exit = None  # exited_process_at of the last traced frame

    def close(self):
        for s in self._scenes.values():
            s.close()
        self._scenes.clear()
        self.ctx.close()

    def _scene(self, project: Path) -> Scene:
        key = str(project)
        s = self._scenes.get(key)
        if s is None:
            scene_file = scene_path_for_project(project, [self.base_directory_path / "scenes"])
            if not scene_file.is_file():
                raise RenderError(f"No exported scene for project {project!s}: expected {scene_file!s} "
                                  "(export it once with tools/blend_export.py)")
            s = self.ctx.load_scene(str(scene_file))
            self._scenes[key] = s
        return s

    def _prepare(self, job: BlenderJob, frame_index: int):
        """Path resolution, checks and output naming of runner/mod.rs:72-139."""
        try:
            blend = parse_with_base_directory_prefix(job.project_file_path, self.base_directory_path)
            script = parse_with_base_directory_prefix(job.render_script_path, self.base_directory_path)
            out_dir = parse_with_base_directory_prefix(job.output_directory_path, self.base_directory_path)
        except JobError as e:
            raise RenderError(str(e)) from e
        if not blend.is_file():
            raise RenderError(f"Invalid blender project file path: file doesn't exist: {str(blend)!r}")
        if not script.is_file():
            # the reference's message names the project path here (runner/mod.rs:99-104)
            raise RenderError(f"Invalid render script: file doesn't exist: {str(blend)!r}")
        if not out_dir.is_dir():
            try:
                out_dir.mkdir(parents=True, exist_ok=True)
            except OSError as e:
                raise RenderError("Could not create missing directories.") from e
        if job.output_file_format not in EXTENSIONS:
            raise RenderError(f"Unsupported output file format {job.output_file_format!r}")
        out_no_ext = output_path_without_extension(str(out_dir), job.output_file_name_format, frame_index)
        return blend, out_no_ext

    def render_frame(self, job: BlenderJob, frame_index: int) -> FrameRenderTime:
        blend, out_no_ext = self._prepare(job, frame_index)
        with self._lock:
            scene = self._scene(blend)
            started_process_at = time.time()
            timing, stats = self.ctx.render_frame(scene, frame_index, self.params, out_no_ext,
                                                  job.output_file_format, 90)
            exited_process_at = time.time()
            frt = self._trace(frame_index, started_process_at, timing, exited_process_at)
        self.last_stats = stats
        return frt

    def _trace(self, frame_index: int, started_process_at: float, timing, exited_process_at: float):
        # a frame's record never starts before the previous one's exit (frames
        # submitted while the previous one was in flight; traces.FrameRenderTime)
        frt = FrameRenderTime.from_timing(started_process_at, timing, exited_process_at, not_before=self._last_exit)
        self._last_exit = frt.exited_process_at
        self.tracer.trace_new_rendered_frame(frame_index, frt)
        return frt

    # Two-phase form (rr_frame_submit / rr_frame_complete): the worker keeps its
    # next queued frame in flight while the previous one is encoded and
    # written. Calls must come from one thread (the queue's), in order.
    def submit_frame(self, job: BlenderJob, frame_index: int) -> "PendingFrame":
        blend, out_no_ext = self._prepare(job, frame_index)
        scene = self._scene(blend)
        t0 = time.time()
        ticket = self.ctx.submit_frame(scene, frame_index, self.params, out_no_ext, job.output_file_format, 90)
        return PendingFrame(frame_index, ticket, t0)

    def complete_frame(self, pending: "PendingFrame"):
        """(FrameRenderTime, stats) of a submitted frame; traced once."""
        try:
            timing, stats = self.ctx.complete_frame(pending.ticket)
        finally:
            pending.done = True
        frt = self._trace(pending.frame_index, pending.started_process_at, timing, time.time())
        self.last_stats = stats
        return frt, stats

    def render_frames(self, job: BlenderJob, frame_indices, on_frame=None) -> list:
        """Render a worker's queued frames in order with frames N+1 and N+2's
        device work in flight while frame N is encoded and written (SURVEY.md
        §8f rank 2; RR_MAX_FRAMES_IN_FLIGHT pending at most). Every frame still gets its own file, FrameRenderTime and
        trace entry, exactly as render_frame would produce them; on_frame
        (frame_index, frt, stats) is called as each one completes."""
        frames = list(frame_indices)
        out = []
        with self._lock:
            pending: deque = deque()

            def retire():
                pf = pending.popleft()
                frt, stats = self.complete_frame(pf)
                out.append(frt)
                if on_frame is not None:
                    on_frame(pf.frame_index, frt, stats)

            try:
                for f in frames:
                    pending.append(self.submit_frame(job, f))
                    if len(pending) >= RR_MAX_FRAMES_IN_FLIGHT:
                        retire()
                while pending:
                    retire()
            finally:
                while pending:  # an error above: drain what is still in flight
                    pf = pending.popleft()
                    try:
                        self.ctx.complete_frame(pf.ticket)
                    except Exception:
                        pass
        return out


class PendingFrame:
    """A frame between submit_frame and complete_frame."""

    def __init__(self, frame_index: int, ticket: int, started_process_at: float):
        self.frame_index = frame_index
        self.ticket = ticket
        self.started_process_at = started_process_at
        self.done = False


class WorkerFrameState(enum.Enum):
    """worker/src/rendering/queue.rs:17-23."""
    QUEUED = "queued"
    RENDERING = "rendering"
    FINISHED = "finished"


class FrameQueueRemoveResult(enum.Enum):
    """shared::messages::queue::FrameQueueRemoveResult (serde names of the reference)."""
    REMOVED_FROM_QUEUE = "removed-from-queue"
    ALREADY_RENDERING = "already-rendering"
    ALREADY_FINISHED = "already-finished"
    ERRORED = "errored"


@dataclass
class WorkerQueueFrame:
    job: BlenderJob
    frame_index: int
    state: WorkerFrameState = WorkerFrameState.QUEUED


class WorkerAutomaticQueue:
    """Mirror of the worker's frame queue (worker/src/rendering/queue.rs:42-229)
    over a runner with submit_frame / complete_frame (BackendRunner).

    Same observable semantics as the reference: frames are queued in order,
    rendered first-queued-first, a frame is RENDERING from the moment its
    render starts until it is removed after completion; a successful frame is
    reported through `on_finished(job_name, frame_index)` (the reference sends
    WorkerFrameQueueItemFinishedEvent::new_ok, queue.rs:144-167), a failed one
    is only logged (queue.rs:169-174); unqueue_frame (the master's steal)
    returns AlreadyRendering / AlreadyFinished / RemovedFromQueue / Errored as
    queue.rs:198-229 does.

    Two differences, neither visible in the protocol:
      * no 100 ms poll (queue.rs:81): queue_frame wakes the loop through a
        condition variable, so a GPU frame of a few ms is not padded to 100 ms;
      * up to `frames_in_flight` (default 2, at most RR_MAX_FRAMES_IN_FLIGHT)
        frames render at once: frame N+1 is
        submitted before frame N is completed, so N's encode and file write
        overlap N+1's device work. N+1 is marked RENDERING when it is
        SUBMITTED (under the queue lock, before the device call), so a steal
        of it returns AlreadyRendering and it can never be both rendered here
        and handed to another worker.
    The connection layer (worker/src/connection/mod.rs:623-656) still owns the
    trace counters (trace_new_frame_queued, trace_frame_stolen_from_queue).
    """

    def __init__(self, runner, on_finished=None, frames_in_flight: int = 2, logger=None):
        if not 1 <= frames_in_flight <= RR_MAX_FRAMES_IN_FLIGHT:
            raise ValueError(f"frames_in_flight must be 1..{RR_MAX_FRAMES_IN_FLIGHT}")
        self.runner = runner
        self.on_finished = on_finished
        self.depth = frames_in_flight
        self.errors: list = []  # (frame_index, exception) of failed renders (logged, not reported)
        self._log = logger
        self._frames: list[WorkerQueueFrame] = []
        self._cv = threading.Condition()
        self._cancel = False
        self._thread = threading.Thread(target=self._run, name="rr-worker-queue", daemon=True)
        self._thread.start()

    # -- the reference's public surface ------------------------------------
    def queue_frame(self, job: BlenderJob, frame_index: int) -> None:
        with self._cv:
            self._frames.append(WorkerQueueFrame(job, int(frame_index)))
            self._cv.notify_all()

    def unqueue_frame(self, job_name: str, frame_index: int):
        """(FrameQueueRemoveResult, reason or None)."""
        with self._cv:
            for i, f in enumerate(self._frames):
                if f.job.job_name == job_name and f.frame_index == frame_index:
                    if f.state is WorkerFrameState.RENDERING:
                        return FrameQueueRemoveResult.ALREADY_RENDERING, None
                    if f.state is WorkerFrameState.FINISHED:
                        return FrameQueueRemoveResult.ALREADY_FINISHED, None
                    del self._frames[i]
                    return FrameQueueRemoveResult.REMOVED_FROM_QUEUE, None
            return FrameQueueRemoveResult.ERRORED, "Can't find such queued frame."

    def cancel(self) -> None:
        """The global cancellation token (queue.rs:83-86): stop taking frames;
        frames already in flight are completed first."""
        with self._cv:
            self._cancel = True
            self._cv.notify_all()

    def join(self, timeout: float | None = None) -> None:
        self._thread.join(timeout)

    def wait_idle(self, timeout: float | None = None) -> bool:
        """Block until no frame is queued or rendering (tests, job end)."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while self._frames:
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return False
                self._cv.wait(left)
        return True

    def states(self) -> list:
        with self._cv:
            return [(f.frame_index, f.state) for f in self._frames]

    # -- the loop ----------------------------------------------------------
    def _next_queued(self):
        for f in self._frames:
            if f.state is WorkerFrameState.QUEUED:
                return f
        return None

    def _finish(self, frame: WorkerQueueFrame, error: Exception | None) -> None:
        if error is None:
            if self.on_finished is not None:
                self.on_finished(frame.job.job_name, frame.frame_index)
        else:
            self.errors.append((frame.frame_index, error))
            if self._log is not None:
                self._log(f"Frame failed to render! {error!r}")
        with self._cv:
            for i, f in enumerate(self._frames):
                if f is frame:
                    del self._frames[i]
                    break
            self._cv.notify_all()

    def _run(self) -> None:
        pending: deque = deque()  # (WorkerQueueFrame, PendingFrame)
        while True:
            with self._cv:
                while not self._cancel and not pending and self._next_queued() is None:
                    self._cv.wait()
                if self._cancel and not pending:
                    return
                nxt = None
                if not self._cancel and len(pending) < self.depth:
                    nxt = self._next_queued()
                    if nxt is not None:
                        nxt.state = WorkerFrameState.RENDERING  # before the render starts: steals see it
            if nxt is not None:
                try:
                    pending.append((nxt, self.runner.submit_frame(nxt.job, nxt.frame_index)))
                except Exception as e:  # noqa: BLE001 - the reference logs and drops the frame
                    self._finish(nxt, e)
                continue
            frame, pf = pending.popleft()
            try:
                self.runner.complete_frame(pf)
                err = None
            except Exception as e:  # noqa: BLE001
                err = e
            self._finish(frame, err)
