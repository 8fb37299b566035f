"""MI355X-native per-frame renderer for the distributed render cluster.

Replaces the one data-parallel hot path of
simongoricar/diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster:
the worker's per-frame render step (a Blender Cycles CPU subprocess in the
reference, /root/reference/worker/src/rendering/runner/mod.rs:72-203) with an
in-process C-ABI call into hand-written CDNA4 HIP kernels (LBVH build +
wavefront path tracer), see DESIGN.md.

Import with importlib (the directory name is not a Python identifier):
    rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")
"""
from .jobs import BlenderJob, DistributionStrategy, JobError, parse_with_base_directory_prefix, \
    scene_path_for_project
from .naming import EXTENSIONS, format_hash_frame_placeholders, job_output_files, output_file_path, \
    output_path_without_extension
from .native import (LIB_PATH, SHIM_PATH, EXPORTS, FrameState, FrameStats, FrameTiming, RenderContext,
                     RenderParams, RRError, Scene, default_params, encode_image, lib)
from .runner import (BackendRunner, FrameQueueRemoveResult, PendingFrame, RenderError, WorkerAutomaticQueue,
                     WorkerFrameState)
from .traces import FrameRenderTime, WorkerTrace, WorkerTraceBuilder, raw_trace_document, save_raw_traces, \
    worker_name

__all__ = [n for n in dir() if not n.startswith("_")]
