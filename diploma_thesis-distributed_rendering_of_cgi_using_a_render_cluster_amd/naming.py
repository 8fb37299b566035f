"""Output file naming of a rendered frame.

Restates /root/reference/scripts/render-timing-script.py:69-78 (hash
substitution) and the path assembly of BlenderJobRunner::render_frame
(/root/reference/worker/src/rendering/runner/mod.rs:111-136: output dir + '/' +
output_file_name_format), plus Blender's write_still extension (R_EXTENSION is
set in the 01 project): ".jpg" for JPEG, ".png" for PNG.
"""
from __future__ import annotations

EXTENSIONS = {"JPEG": ".jpg", "PNG": ".png"}


def format_hash_frame_placeholders(raw_file_path: str, frame_number: int) -> str:
    """Count every '#' in the path, then replace each run of exactly that many
    '#' with the frame number zero-padded to that width (never truncated).
    With no '#' at all the reference replaces the EMPTY string, i.e. inserts
    the frame number between every character (tests/golden/naming.json)."""
    n = raw_file_path.count("#")
    return raw_file_path.replace("#" * n, str(frame_number).rjust(n, "0"))


def output_path_without_extension(output_directory: str, name_format: str, frame_number: int) -> str:
    # The whole path goes through the substitution, directory included, exactly
    # as the reference passes "<dir>/<fmt>" as --render-output (runner/mod.rs:124-127).
    return format_hash_frame_placeholders(output_directory + "/" + name_format, frame_number)


def output_file_path(output_directory: str, name_format: str, frame_number: int, file_format: str) -> str:
    if file_format not in EXTENSIONS:
        raise ValueError(f"unsupported output format {file_format!r}")
    return output_path_without_extension(output_directory, name_format, frame_number) + EXTENSIONS[file_format]


def job_output_files(job, output_directory: str) -> list[str]:
    """Every file a job writes (frame set from..=to, master/src/cluster/state.rs:51-53)."""
    return [output_file_path(output_directory, job.output_file_name_format, f, job.output_file_format)
            for f in job.frames()]
