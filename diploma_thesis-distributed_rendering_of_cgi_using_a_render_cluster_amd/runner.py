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
The Rust worker's equivalent (spawn_blocking over the same C ABI) is in
INTEGRATION.md; this Python class is what the tests and bench.py drive.
"""
from __future__ import annotations

import os
import threading
import time
from pathlib import Path

from .jobs import BlenderJob, JobError, parse_with_base_directory_prefix, scene_path_for_project
from .naming import EXTENSIONS, output_path_without_extension
from .native import RenderContext, RenderParams, Scene
from .traces import FrameRenderTime, WorkerTraceBuilder


class RenderError(RuntimeError):
    pass


class BackendRunner:
    def __init__(self, base_directory_path: str | os.PathLike, tracer: WorkerTraceBuilder | None = None,
                 device: int = 0, params: RenderParams | None = None):
        base = Path(base_directory_path)
        if not base.is_dir():
            raise RenderError("Provided base directory path is not a directory.")
        self.base_directory_path = base
        self.tracer = tracer if tracer is not None else WorkerTraceBuilder()
        self.params = params
        self.ctx = RenderContext(device)
        self._scenes: dict[str, Scene] = {}
        self._lock = threading.Lock()  # one frame in flight per context (queue.rs:79-118)
        self.last_stats = None

    def close(self):
        for s in self._scenes.values():
            s.close()
        self._scenes.clear()
        self.ctx.close()

    def _scene(self, project: Path) -> Scene:
        key = str(project)
        s = self._scenes.get(key)
        if s is None:
            scene_file = scene_path_for_project(project)
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
        self.last_stats = stats
        frt = FrameRenderTime.from_timing(started_process_at, timing, exited_process_at)
        self.tracer.trace_new_rendered_frame(frame_index, frt)
        return frt

    def render_frames(self, job: BlenderJob, frame_indices, on_frame=None) -> list:
        """Render a worker's queued frames in order with frame N+1's device
        work in flight while frame N is encoded and written (rr_frame_submit /
        rr_frame_complete). Every frame still gets its own
        file, FrameRenderTime and trace entry, exactly as render_frame would
        produce them; on_frame(frame_index, frt, stats) is called as each one
        completes. started_process_at is the frame's submit time."""
        frames = list(frame_indices)
        out = []
        with self._lock:
            pending = []  # (frame, ticket, started_process_at)

            def retire():
                f, t, t0 = pending.pop(0)
                timing, stats = self.ctx.complete_frame(t)
                frt = FrameRenderTime.from_timing(t0, timing, time.time())
                self.last_stats = stats
                self.tracer.trace_new_rendered_frame(f, frt)
                out.append(frt)
                if on_frame is not None:
                    on_frame(f, frt, stats)

            try:
                for f in frames:
                    blend, out_no_ext = self._prepare(job, f)
                    scene = self._scene(blend)
                    t0 = time.time()
                    ticket = self.ctx.submit_frame(scene, f, self.params, out_no_ext, job.output_file_format, 90)
                    pending.append((f, ticket, t0))
                    if len(pending) >= 2:
                        retire()
                while pending:
                    retire()
            finally:
                while pending:  # an error above: drain what is still in flight
                    f, t, _ = pending.pop(0)
                    try:
                        self.ctx.complete_frame(t)
                    except Exception:
                        pass
        return out
