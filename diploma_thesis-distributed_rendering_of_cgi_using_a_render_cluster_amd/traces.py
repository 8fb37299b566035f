"""Worker trace records — the output record of the per-frame render step.

Mirrors shared::results::worker_trace (/root/reference/shared/src/results/worker_trace.rs):
FrameRenderTime (:13-45, seven DateTime<Utc> serialised as
TimestampSecondsWithFrac<f64>), WorkerFrameTrace (:47-62), ping and
reconnection traces (:64-100), WorkerTrace (:103-126) and WorkerTraceBuilder
(:150-236); plus the raw-trace file the master writes
(/root/reference/master/src/main.rs:43-96), which analysis/ consumes.
"""
from __future__ import annotations

import json
import math
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path

FRAME_FIELDS = ("started_process_at", "finished_loading_at", "started_rendering_at", "finished_rendering_at",
                "file_saving_started_at", "file_saving_finished_at", "exited_process_at")


def as_utc_seconds(t: float) -> float:
    """f64 seconds -> DateTime<Utc> -> f64, as the reference round-trips them:
    whole seconds plus nanoseconds truncated (utilities.rs:86-96)."""
    whole = math.floor(t)
    ns = int((t - whole) * 1e9)
    return whole + ns / 1e9


@dataclass(frozen=True)
class FrameRenderTime:
    started_process_at: float
    finished_loading_at: float
    started_rendering_at: float
    finished_rendering_at: float
    file_saving_started_at: float
    file_saving_finished_at: float
    exited_process_at: float

    @classmethod
    def from_timing(cls, started_process_at: float, timing, exited_process_at: float,
                    not_before: float | None = None) -> "FrameRenderTime":
        """PartialRenderStatistics::with_process_information (utilities.rs:23-37).

        not_before: exited_process_at of the worker's previous frame when this
        frame was submitted while that one was still in flight (two frames in
        flight, BackendRunner.render_frames / WorkerAutomaticQueue). The
        reference's per-worker accounting (WorkerPerformance::from_worker_trace,
        shared/src/results/performance.rs:70-130) needs consecutive frames
        that do not overlap: idle = started_process_at - previous
        exited_process_at must not be negative (`to_std()` fails otherwise).
        The frame's record therefore starts when the previous one ended, and
        every later timestamp is kept at or after its predecessor, so the seven
        stay ordered."""
        vals = [as_utc_seconds(v) for v in (started_process_at, timing.loaded_at, timing.started_rendering_at,
                                             timing.finished_rendering_at, timing.file_saving_started_at,
                                             timing.file_saving_finished_at, exited_process_at)]
        if not_before is not None:  # compared as serialised (truncated) values: equal floats, zero idle
            vals[0] = max(vals[0], not_before)
            for k in range(1, len(vals)):
                vals[k] = max(vals[k], vals[k - 1])
        return cls(*vals)

    def total_execution_time(self) -> float:
        d = self.exited_process_at - self.started_process_at
        if d < 0:
            raise ValueError("Total execution time is negative?!")
        return d

    def to_dict(self) -> dict:
        return {k: getattr(self, k) for k in FRAME_FIELDS}


@dataclass
class WorkerTrace:
    total_queued_frames: int
    total_queued_frames_removed_from_queue: int
    job_start_time: float
    job_finish_time: float
    frame_render_traces: list = field(default_factory=list)  # [(frame_index, FrameRenderTime)]
    ping_traces: list = field(default_factory=list)          # [(pinged_at, received_at)]
    reconnection_traces: list = field(default_factory=list)  # [(lost_connection_at, reconnected_at)]

    def to_dict(self) -> dict:
        return {
            "total_queued_frames": self.total_queued_frames,
            "total_queued_frames_removed_from_queue": self.total_queued_frames_removed_from_queue,
            "job_start_time": self.job_start_time,
            "job_finish_time": self.job_finish_time,
            "frame_render_traces": [{"frame_index": i, "details": f.to_dict()} for i, f in self.frame_render_traces],
            "ping_traces": [{"pinged_at": a, "received_at": b} for a, b in self.ping_traces],
            "reconnection_traces": [{"lost_connection_at": a, "reconnected_at": b}
                                    for a, b in self.reconnection_traces],
        }


class WorkerTraceBuilder:
    """Thread-safe builder (the reference wraps it in Arc<Mutex<…>>)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._queued = 0
        self._removed = 0
        self._start = None
        self._finish = None
        self._frames = []
        self._pings = []
        self._reconnects = []

    def trace_new_frame_queued(self):
        with self._lock:
            self._queued += 1

    def trace_frame_stolen_from_queue(self):
        with self._lock:
            self._removed += 1

    def set_job_start_time(self, t: float):
        with self._lock:
            self._start = as_utc_seconds(t)

    def set_job_finish_time(self, t: float):
        with self._lock:
            self._finish = as_utc_seconds(t)

    def trace_new_rendered_frame(self, frame_index: int, frt: FrameRenderTime):
        with self._lock:
            self._frames.append((int(frame_index), frt))

    def trace_new_ping(self, pinged_at: float, received_at: float):
        with self._lock:
            self._pings.append((as_utc_seconds(pinged_at), as_utc_seconds(received_at)))

    def trace_new_reconnect(self, lost: float, reconnected: float):
        with self._lock:
            self._reconnects.append((as_utc_seconds(lost), as_utc_seconds(reconnected)))

    def frames(self) -> list:
        with self._lock:
            return list(self._frames)

    def build(self) -> WorkerTrace:
        with self._lock:
            if self._start is None:
                raise ValueError("Missing job start time, can't build.")
            if self._finish is None:
                raise ValueError("Missing job finish time, can't build.")
            return WorkerTrace(self._queued, self._removed, self._start, self._finish, list(self._frames),
                               list(self._pings), list(self._reconnects))


def raw_trace_document(job, master_start: float, master_finish: float, worker_traces: dict) -> dict:
    """RawTraceWrapper {job, master_trace, worker_traces} (master/src/main.rs:43-47)."""
    return {"job": job.to_dict(),
            "master_trace": {"job_start_time": as_utc_seconds(master_start),
                             "job_finish_time": as_utc_seconds(master_finish)},
            "worker_traces": {k: v.to_dict() for k, v in worker_traces.items()}}


def save_raw_traces(job, output_directory: str | Path, master_start: float, master_finish: float,
                    worker_traces: dict, start_local: float | None = None) -> Path:
    """Writes <YYYY-mm-dd_HH-MM-SS>_job-<name>_raw-trace.json (master/src/main.rs:49-96)."""
    out = Path(output_directory)
    out.mkdir(parents=True, exist_ok=True)
    stamp = time.strftime("%Y-%m-%d_%H-%M-%S", time.localtime(start_local if start_local else master_start))
    path = out / f"{stamp}_job-{job.job_name.replace(' ', '_')}_raw-trace.json"
    path.write_text(json.dumps(raw_trace_document(job, master_start, master_finish, worker_traces), indent=2))
    return path


def worker_name(worker_id: int, address: str) -> str:
    """Key of worker_traces: "<8 hex digits of the worker id>-<ip:port>"."""
    return f"{worker_id & 0xFFFFFFFF:08x}-{address}"
