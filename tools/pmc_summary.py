#!/usr/bin/env python3
"""Per-kernel summaries of rocprofv3 output directories (CSV format), written
into profiles/ so bench.py can quote PMC-measured HBM traffic per launch.

  python tools/pmc_summary.py stats  <kernel-trace dir> > profiles/r1_kernel_stats.md
  python tools/pmc_summary.py traffic --fetch <dir> --write <dir> [--sq <dir> ...] -o profiles/r1_pmc.json

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB.
On gfx950 FETCH_SIZE counts 64 B per TCC read request whatever its size:
tools/fetch_probe.hip measured 0.500 FETCH_SIZE bytes per byte read for a
coalesced 16 B/lane stream (128 B requests) and 1.000 for random 64 B node
gathers (profiles/r4_fetch_probe.json). So the read bytes are 2 x FETCH_SIZE x
1024 for streaming kernels and FETCH_SIZE x 1024 for the traversal kernels,
whose reads are 64 B node and triangle fetches (GATHER below); the raw value
and the other bound are kept beside it.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

_NAME = re.compile(r"(k_\w+)(<[^>(]*>)?")
# kernels whose reads are 64 B gathers (FETCH_SIZE x 1 per the probe)
GATHER = ("k_trace_primary", "k_trace_extend", "k_shadow_refill", "k_trace_primary_packet")


def short_name(full: str) -> str:
    m = _NAME.search(full)
    if not m:
        return full.split("(")[0][-60:]
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def _rows(d: str, suffix: str):
    files = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not files:
        raise SystemExit(f"no *{suffix} under {d}")
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def kernel_stats(d: str) -> dict:
    out = {}
    for r in _rows(d, "kernel_stats.csv"):
        out[short_name(r["Name"])] = {"calls": int(r["Calls"]), "total_ms": int(r["TotalDurationNs"]) / 1e6,
                                      "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])}
    return out


def counters(d: str) -> dict:
    """{kernel: {counter: [per-dispatch values]}} from a --pmc pass."""
    acc = defaultdict(lambda: defaultdict(dict))
    for r in _rows(d, "counter_collection.csv"):
        k = short_name(r["Kernel_Name"])
        acc[k][r["Counter_Name"]][r.get("Dispatch_Id") or r.get("Correlation_Id")] = float(r["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in acc.items()}


def cmd_stats(a):
    st = kernel_stats(a.dir)
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---:|---:|---:|---:|")
    for k, v in sorted(st.items(), key=lambda kv: -kv[1]["total_ms"]):
        print(f"| `{k}` | {v['calls']} | {v['total_ms']:.3f} | {v['avg_ms']:.4f} | {v['pct']:.2f} |")


def pass_durations(d: str) -> dict:
    """{kernel: mean dispatch ns} from the kernel trace of a --pmc pass run with
    --kernel-trace (empty if the pass has none)."""
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                acc[short_name(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def cmd_traffic(a):
    fetch, write = counters(a.fetch), counters(a.write)
    extra, durs = {}, {}
    for d in a.sq or []:
        cs_d = counters(d)
        dur = pass_durations(d)
        for k, cs in cs_d.items():
            extra.setdefault(k, {}).update(cs)
            # the counting pass's own dispatch durations (profiler-serialised, so
            # not the bench's launch time; reported for reference). No clock is
            # derived from GRBM_GUI_ACTIVE here: it counts GPU-busy cycles of a
            # clock domain whose rate and per-XCD summation are not pinned, and
            # the quotient came out above the 2.4 GHz peak engine clock.
            if k in dur:
                durs[k] = {"pmc_pass_avg_ms": dur[k] / 1e6}
    out = {"source": {"fetch": a.fetch, "write": a.write, "sq": a.sq or []},
           "units": "bytes per launch; fetch_bytes = 2 x FETCH_SIZE(KiB) x 1024 for streaming kernels, "
                    "1 x for the traversal kernels (64 B gathers; tools/fetch_probe.hip calibration)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("FETCH_SIZE", [])
        w = write.get(k, {}).get("WRITE_SIZE", [])
        n = max(len(f), len(w), 1)
        fr = sum(f) / max(len(f), 1) * 1024.0
        wr = sum(w) / max(len(w), 1) * 1024.0
        scale = 1.0 if k.split("<")[0] in GATHER else 2.0
        e = {"launches": n, "fetch_size_raw_bytes": fr, "fetch_scale": scale, "fetch_bytes": scale * fr,
             "fetch_bytes_if_streaming": 2.0 * fr, "write_bytes": wr, "traffic_bytes": scale * fr + wr}
        for c, vals in extra.get(k, {}).items():
            e[c] = sum(vals) / max(len(vals), 1)
        e.update(durs.get(k, {}))
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e and e["TCC_HIT_sum"] + e["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = e["TCC_HIT_sum"] / (e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        if "SQ_WAIT_ANY" in e and e.get("SQ_WAVE_CYCLES", 0) > 0:
            e["wait_frac"] = e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"]
        # active lanes per VALU instruction (rocprofiler-sdk counter_defs.yaml
        # VALUUtilization: THREAD_CYCLES_VALU / (ACTIVE_INST_VALU x wave size));
        # SQ_INSTS_VALU counts wave-instructions whatever the exec mask
        if e.get("SQ_ACTIVE_INST_VALU", 0) > 0 and "SQ_THREAD_CYCLES_VALU" in e:
            e["valu_lane_util"] = e["SQ_THREAD_CYCLES_VALU"] / (64.0 * e["SQ_ACTIVE_INST_VALU"])
        out["kernels"][k] = e
    with open(a.o, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: round(v["traffic_bytes"] / 1e6, 3) for k, v in out["kernels"].items()}))


def main(argv=None):
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("stats")
    s.add_argument("dir")
    t = sub.add_parser("traffic")
    t.add_argument("--fetch", required=True)
    t.add_argument("--write", required=True)
    t.add_argument("--sq", action="append")
    t.add_argument("-o", required=True)
    a = ap.parse_args(argv)
    {"stats": cmd_stats, "traffic": cmd_traffic}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
