#!/usr/bin/env python3
"""Calibrates the PMC byte counters against kernels of known traffic
(tools/fetch_probe.hip): per kernel, FETCH_SIZE (KiB) x 1024 over the bytes
the kernel must read, and the TCC read-request counters per 64 B it must read
(FETCH_SIZE = (TCC_BUBBLE x 128 + (RDREQ - BUBBLE - RDREQ_32B) x 64 +
RDREQ_32B x 32) / 1024 on gfx950, rocprofiler-sdk counter_defs.yaml), from
rocprofv3 --pmc output directories.
  python tools/fetch_probe.py <probe stdout json> <pmc dir> [<pmc dir> ...]"""
import csv
import glob
import json
import os
import sys


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                out.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return out


def main():
    known = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    res = {"known": known, "kernels": {}}
    for d in sys.argv[2:]:
        for k, cs in counters(d).items():
            e = res["kernels"].setdefault(k, {})
            for c, vals in cs.items():
                e[c] = sum(vals) / len(vals)
    for k, e in res["kernels"].items():
        b = known["stream_bytes_per_launch"] if "stream" in k else known["gather_bytes_per_launch"]
        if "FETCH_SIZE" in e:
            e["fetch_size_bytes_over_known"] = e["FETCH_SIZE"] * 1024.0 / b
        for c in ("TCC_EA0_RDREQ_sum", "TCC_BUBBLE_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_DRAM_sum"):
            if c in e:
                e[c + "_per_known_64B"] = e[c] / (b / 64.0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
