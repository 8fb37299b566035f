"""Job descriptor — the input type of the per-frame render step.

Mirrors shared::jobs (/root/reference/shared/src/jobs/mod.rs): the BlenderJob
TOML schema (:45-81), DistributionStrategy with serde tag `strategy_type`
(:32-43) and DynamicStrategyOptions (:8-30), BlenderJob::load_from_file
(:84-100), plus worker::utilities::parse_with_base_directory_prefix
(/root/reference/worker/src/utilities.rs:5-21). serde semantics kept: every
non-Option field is required, unknown keys are ignored, strategy_type must be
one of the three serde names.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

try:
    import tomllib as _toml  # Python >= 3.11
except ModuleNotFoundError:  # pragma: no cover - 3.10 image
    import tomli as _toml


class JobError(ValueError):
    pass


STRATEGIES = ("naive-fine", "eager-naive-coarse", "dynamic")


@dataclass(frozen=True)
class DistributionStrategy:
    strategy_type: str
    target_queue_size: int | None = None
    min_queue_size_to_steal: int | None = None
    min_seconds_before_resteal_to_elsewhere: int | None = None
    min_seconds_before_resteal_to_original_worker: int | None = None

    @classmethod
    def from_dict(cls, d: dict) -> "DistributionStrategy":
        if not isinstance(d, dict) or "strategy_type" not in d:
            raise JobError("frame_distribution_strategy: missing field `strategy_type`")
        t = d["strategy_type"]
        if t not in STRATEGIES:
            raise JobError(f"frame_distribution_strategy: unknown variant `{t}`, expected one of "
                           + ", ".join(f"`{s}`" for s in STRATEGIES))
        need = {"naive-fine": [], "eager-naive-coarse": ["target_queue_size"],
                "dynamic": ["target_queue_size", "min_queue_size_to_steal",
                            "min_seconds_before_resteal_to_elsewhere",
                            "min_seconds_before_resteal_to_original_worker"]}[t]
        vals = {}
        for k in need:
            if k not in d:
                raise JobError(f"frame_distribution_strategy: missing field `{k}`")
            v = d[k]
            if not isinstance(v, int) or isinstance(v, bool) or v < 0:
                raise JobError(f"frame_distribution_strategy: `{k}` must be a usize")
            vals[k] = v
        return cls(t, **vals)

    def to_dict(self) -> dict:
        out = {"strategy_type": self.strategy_type}
        for k in ("target_queue_size", "min_queue_size_to_steal", "min_seconds_before_resteal_to_elsewhere",
                  "min_seconds_before_resteal_to_original_worker"):
            v = getattr(self, k)
            if v is not None:
                out[k] = v
        return out


@dataclass(frozen=True)
class BlenderJob:
    job_name: str
    job_description: str | None
    project_file_path: str
    render_script_path: str
    frame_range_from: int
    frame_range_to: int
    wait_for_number_of_workers: int
    frame_distribution_strategy: DistributionStrategy
    output_directory_path: str
    output_file_name_format: str
    output_file_format: str
    extra: dict = field(default_factory=dict, compare=False, repr=False)

    _STR = ("job_name", "project_file_path", "render_script_path", "output_directory_path",
            "output_file_name_format", "output_file_format")
    _USIZE = ("frame_range_from", "frame_range_to", "wait_for_number_of_workers")

    @classmethod
    def from_dict(cls, d: dict) -> "BlenderJob":
        vals = {}
        for k in cls._STR:
            if k not in d:
                raise JobError(f"missing field `{k}`")
            if not isinstance(d[k], str):
                raise JobError(f"invalid type for `{k}`: expected a string")
            vals[k] = d[k]
        for k in cls._USIZE:
            if k not in d:
                raise JobError(f"missing field `{k}`")
            v = d[k]
            if not isinstance(v, int) or isinstance(v, bool) or v < 0:
                raise JobError(f"invalid value for `{k}`: expected usize")
            vals[k] = v
        desc = d.get("job_description")
        if desc is not None and not isinstance(desc, str):
            raise JobError("invalid type for `job_description`")
        if "frame_distribution_strategy" not in d:
            raise JobError("missing field `frame_distribution_strategy`")
        strat = DistributionStrategy.from_dict(d["frame_distribution_strategy"])
        extra = {k: v for k, v in d.items() if k not in cls._STR + cls._USIZE
                 + ("job_description", "frame_distribution_strategy")}
        return cls(job_description=desc, frame_distribution_strategy=strat, extra=extra, **vals)

    @classmethod
    def load_from_file(cls, path: str | os.PathLike) -> "BlenderJob":
        p = Path(path)
        if p.exists() and not p.is_file():
            raise JobError("Path exists, but it is not a file!")
        if not p.exists():
            raise JobError("No such file!")
        try:
            with open(p, "rb") as f:
                data = _toml.load(f)
        except _toml.TOMLDecodeError as e:
            raise JobError(f"Could not parse TOML contents of job file: {e}") from e
        return cls.from_dict(data)

    def frames(self) -> list[int]:
        """Frame set of the job (master/src/cluster/state.rs:51-53: from..=to)."""
        return list(range(self.frame_range_from, self.frame_range_to + 1))

    def to_dict(self) -> dict:
        """serde_json shape of BlenderJob (field order as the Rust struct)."""
        return {"job_name": self.job_name, "job_description": self.job_description,
                "project_file_path": self.project_file_path, "render_script_path": self.render_script_path,
                "frame_range_from": self.frame_range_from, "frame_range_to": self.frame_range_to,
                "wait_for_number_of_workers": self.wait_for_number_of_workers,
                "frame_distribution_strategy": self.frame_distribution_strategy.to_dict(),
                "output_directory_path": self.output_directory_path,
                "output_file_name_format": self.output_file_name_format,
                "output_file_format": self.output_file_format}


def parse_with_base_directory_prefix(path: str, base: str | os.PathLike | None) -> Path:
    """worker/src/utilities.rs:5-21: a leading %BASE% is replaced by the base
    directory (one leading '/' then one leading '\\' stripped from the rest)."""
    if path.startswith("%BASE%"):
        if base is None:
            raise JobError("Missing base!")
        rest = path[len("%BASE%"):]
        if rest.startswith("/"):
            rest = rest[1:]
        if rest.startswith("\\"):
            rest = rest[1:]
        return Path(base) / rest
    return Path(path)


def scene_path_for_project(project_file: Path, scene_dirs=()) -> Path:
    """The exported scene of a project (tools/blend_export.py writes it once per
    project): <stem>.rrscene next to the .blend, else the first
    <dir>/<stem>.rrscene of scene_dirs that exists (BackendRunner passes the
    base directory's scenes/, where this repository keeps its exports). A
    .rrscene project names itself."""
    p = Path(project_file)
    if p.suffix == ".rrscene":
        return p
    here = p.with_suffix(".rrscene")
    if here.is_file():
        return here
    for d in scene_dirs:
        q = Path(d) / (p.stem + ".rrscene")
        if q.is_file():
            return q
    return here
