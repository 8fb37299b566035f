"""Host-side measurement logic of bench.py and tools/pmc_summary.py (CPU only):
the PMC byte calibration per kernel class, the CPU-baseline band sampler, and
the reference master's dispatch ceiling."""
import csv
import json
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import pmc_summary  # noqa: E402


def _counter_dir(tmp, name, rows):
    d = tmp / name
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (k, c, v) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})
    return str(d)


def test_fetch_size_scale_per_kernel_class(tmp_path):
    """FETCH_SIZE counts 64 B per read request on gfx950 (tools/fetch_probe.hip):
    x1 for the traversal kernels' 64 B gathers, x2 for streaming kernels."""
    fetch = _counter_dir(tmp_path, "fetch", [("k_trace_extend<false>(SceneArgs)", "FETCH_SIZE", 1000.0),
                                             ("k_accumulate(FrameConsts)", "FETCH_SIZE", 1000.0)])
    write = _counter_dir(tmp_path, "write", [("k_trace_extend<false>(SceneArgs)", "WRITE_SIZE", 10.0),
                                             ("k_accumulate(FrameConsts)", "WRITE_SIZE", 10.0)])
    out = tmp_path / "pmc.json"
    pmc_summary.main(["traffic", "--fetch", fetch, "--write", write, "-o", str(out)])
    k = json.load(open(out))["kernels"]
    ext, acc = k["k_trace_extend<false>"], k["k_accumulate"]
    assert ext["fetch_scale"] == 1.0 and acc["fetch_scale"] == 2.0
    assert ext["traffic_bytes"] == 1000.0 * 1024 + 10.0 * 1024
    assert acc["traffic_bytes"] == 2000.0 * 1024 + 10.0 * 1024
    assert ext["fetch_bytes_if_streaming"] == acc["fetch_bytes"]


def test_cpu_baseline_bands(monkeypatch):
    """The sizing band is the frame's middle rows; the spread bands cover the
    other rows; a frame done whole is extrapolated from all of it, a sample
    from the spread bands alone."""
    calls = []
    H, W = 64, 8

    def render_state(state, rows, threads, film):
        calls.append(rows)
        return None, None

    fake = types.SimpleNamespace(render_state=render_state, last_build_seconds=lambda: 0.0)
    state = types.SimpleNamespace(render_ints=np.array([W, H, 4], np.int32))
    monkeypatch.setattr(bench, "host_cpu", lambda: (8, 8, "test"))
    r = bench.cpu_baseline(fake, state, 1e9, "test", threads=2)
    assert calls[0] == (32, 36)  # the middle rows first
    covered = sorted(set(y for a, b in calls for y in range(a, b)))
    assert covered == list(range(H))  # whole frame, every row once
    assert sum(b - a for a, b in calls) == H
    assert r["cores"] == 2 and r["value"] > 0 and "row 32" in r["sample"]


def test_dispatch_ceiling_matches_reference_strategies():
    """Frames per second the unchanged master can hand one worker:
    eager-naive-coarse tops the queue up to target_queue_size every 100 ms,
    dynamic every 50 ms, naive-fine one frame per 50 ms
    (master/src/cluster/strategies.rs)."""
    coarse = {"frame_distribution_strategy": {"strategy_type": "eager-naive-coarse", "target_queue_size": 4}}
    dyn = {"frame_distribution_strategy": {"strategy_type": "dynamic", "target_queue_size": 4}}
    fine = {"frame_distribution_strategy": {"strategy_type": "naive-fine"}}
    assert bench.dispatch_ceiling(coarse, 1)["value"] == 40.0
    assert bench.dispatch_ceiling(dyn, 1)["value"] == 80.0
    assert bench.dispatch_ceiling(fine, 1)["value"] == 20.0
    assert bench.dispatch_ceiling(coarse, 8)["value"] == 320.0
