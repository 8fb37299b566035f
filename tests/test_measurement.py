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


def _split_stats(n_tris):
    """Counting-frame stats of a split-path frame (one extension launch)."""
    return types.SimpleNamespace(camera_rays=1000, extension_rays=500, shadow_rays=400, primary_continued=300,
                                 primary_shadow=250, trav_nodes=[1000, 8000, 6000], trav_tris=[100, 900, 700],
                                 n_triangles=n_tris, width=10, height=10, spp=10, chunks=1,
                                 camera_rays_traced=900)


def _roof(tmp_path, entry, n_tris):
    pmc = tmp_path / "pmc.json"
    pmc.write_text(json.dumps({"kernels": {"k_trace_extend<false>": entry}}))
    args = types.SimpleNamespace(workload="c5", pmc_summary=str(pmc))
    names = ["build", "primary", "extend", "shadow", "accumulate", "shade", "tiles", "x"]
    ms, launches = [0.0] * 8, [0] * 8
    ms[2], launches[2], launches[5] = 2.0, 1, 1  # 1 extension launch of 2 ms; a shading launch (split path)
    return bench.roofline_line(args, "extend", _split_stats(n_tris), ms, launches, names, 1)


def test_split_path_bound_comes_from_the_counters(tmp_path):
    """The split path's bound is derived from its PMC pass: latency when the
    PMC HBM rate is below half the peak and waves wait more than half their
    lives, else hbm; frac is the PMC fraction, the SURVEY 8(d) figure beside
    it as frac_survey_formula."""
    slow = {"traffic_bytes": 2e12 * 2.0e-3, "wait_frac": 0.59, "l2_hit_rate": 0.36}  # 2 TB/s
    r = _roof(tmp_path, slow, 10_000_000)
    assert r["bound"] == "latency" and abs(r["achieved"] - 2000.0) < 1e-6
    assert abs(r["frac"] - 0.25) < 1e-9 and "frac_survey_formula" in r
    fast = {"traffic_bytes": 6e12 * 2.0e-3, "wait_frac": 0.7}  # 6 TB/s
    assert _roof(tmp_path, fast, 10_000_000)["bound"] == "hbm"
    busy = {"traffic_bytes": 1e12 * 2.0e-3, "wait_frac": 0.3, "SQ_INSTS_VALU": 614.4e9 * 2.0e-3}
    r = _roof(tmp_path, busy, 1000)  # slow memory, but the waves issue: half the VALU issue peak
    assert r["bound"] == "valu" and r["unit"] == "G wave-instr/s" and abs(r["frac"] - 0.5) < 1e-3
    assert r["hbm_gbs_pmc"] == 1000.0


def test_kernels_pmc_block():
    """Per-kernel PMC rows: the timed instantiation only, GB/s over the pass's
    own dispatch time, wave life and occupancy from SQ_WAVE_CYCLES over that
    dispatch time x the engine clock."""
    span = 2.0e-3 * 2.4e9  # 2 ms at the 2.4 GHz peak clock, in cycles
    ks = {"k_trace_extend<false>": {"launches": 4, "traffic_bytes": 8e9, "pmc_pass_avg_ms": 2.0,
                                    "l2_hit_rate": 0.5, "wait_frac": 0.6, "valu_lane_util": 0.45,
                                    "GRBM_GUI_ACTIVE": 8 * span, "SQ_WAVE_CYCLES": span / 4 * 2048, "SQ_WAVES": 2048},
          "k_trace_extend<true>": {"launches": 1, "traffic_bytes": 1.0, "pmc_pass_avg_ms": 1.0},
          "k_shade_extend": {"launches": 4, "traffic_bytes": 2e9, "pmc_pass_avg_ms": 1.0}}
    b = bench.pmc_kernel_block(ks, "profiles/x.json")
    rows = b["kernels"]
    assert set(rows) == {"k_trace_extend<false>", "k_shade_extend"}
    e = rows["k_trace_extend<false>"]
    assert e["hbm_gbs"] == 4000.0 and e["hbm_frac"] == 0.5
    assert e["wave_life_frac"] == 1.0 and e["occupancy_waves_per_simd"] == 2.0
    assert e["grbm_span_over_dispatch"] == 1.0
    assert rows["k_shade_extend"]["hbm_gbs"] == 2000.0
    assert bench.pmc_kernel_block({}, None) == {}


def test_occupancy_ignores_an_overstated_grbm_span():
    """VERDICT r5 Weak 4: in the pipelined PMC pass GRBM_GUI_ACTIVE / 8 was 3.4x
    k_tiles' dispatch time (other kernels' busy cycles counted), which made its
    occupancy read 0.96 waves/SIMD for a kernel launched at 4. The span is the
    dispatch time x the clock, so the same counters give the launch's real
    figures, and the GRBM ratio is only reported."""
    ms, clock = 1.076, 2.382  # r5 k_tiles<false,false>: dispatch, measured kernel clock
    span = ms * 1e-3 * clock * 1e9
    waves = 4096  # 4 waves per SIMD, all resident from the start
    e = {"launches": 2, "traffic_bytes": 6.9e7, "pmc_pass_avg_ms": ms, "GRBM_GUI_ACTIVE": 8 * 3.4 * span,
         "SQ_WAVES": waves, "SQ_WAVE_CYCLES": 0.8 * span / 4 * waves}  # each wave lives 0.8 of the launch
    occ = bench.occupancy_figures(e, clock)
    assert occ["wave_life_frac"] == 0.8 and occ["occupancy_waves_per_simd"] == 3.2
    assert occ["grbm_span_over_dispatch"] == 3.4
    row = bench.pmc_kernel_block({"k_tiles<false,false>": e}, "x", clock)["kernels"]["k_tiles<false,false>"]
    assert row["occupancy_waves_per_simd"] == 3.2  # the GRBM span would have said 0.94
    assert bench.occupancy_figures({"pmc_pass_avg_ms": 1.0}) == {}
