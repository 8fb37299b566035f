#!/usr/bin/env python3
"""Print one or two frames of a rocprofv3 --kernel-trace [--hip-trace
--memory-copy-trace] csv run: device activity per queue and, if present, the
HIP API calls of the same window (times in us from the window start).
  python tools/trace_timeline.py <dir with run_*_trace.csv> [--kernel k_tiles] [--frames 2]"""
import argparse
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--kernel", default="k_tiles")
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--api-min-us", type=float, default=20.0)
a = ap.parse_args()


def rows(name):
    p = os.path.join(a.dir, name)
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


ev = []
for r in rows("run_kernel_trace.csv"):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K q" + r["Queue_Id"], r["Kernel_Name"][:48],
               r["Correlation_Id"]))
for r in rows("run_memory_copy_trace.csv"):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", r.get("Direction", ""), r["Correlation_Id"]))
ev.sort()
marks = [e for e in ev if a.kernel in e[3]]
lo = marks[-(a.frames + 2)][0]
hi = marks[-2][1]
for e in ev:
    if lo <= e[0] <= hi:
        print(f"{(e[0] - lo) / 1e3:9.1f} {(e[1] - lo) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f} {e[2]:5s} {e[3]} c{e[4]}")
api = [r for r in rows("run_hip_api_trace.csv") if lo <= int(r["Start_Timestamp"]) <= hi]
if api:
    print("--- HIP API")
    for r in sorted(api, key=lambda r: int(r["Start_Timestamp"])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        f = r["Function"]
        if (e - s) / 1e3 >= a.api_min_us or any(k in f for k in ("Memcpy", "Launch", "Synchron")):
            print(f"{(s - lo) / 1e3:9.1f} {(e - lo) / 1e3:9.1f} {(e - s) / 1e3:8.1f} T{r['Thread_Id']} {f} c{r['Correlation_Id']}")
