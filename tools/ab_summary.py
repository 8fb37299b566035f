#!/usr/bin/env python3
"""Summary of tools/ab_run.py output: per scene and variant, the best solo
total over the rounds, the per-class means and the pipelined frames/s.
  python tools/ab_summary.py gpurun_out/abN.txt"""
import collections
import json
import sys


def main():
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for line in open(sys.argv[1]):
        if not line.startswith("r") or "{" not in line:
            if line.strip():
                print(line.rstrip()[:300])
            continue
        _, v, js = line.split(None, 2)
        for sc, x in json.loads(js).items():
            res[sc][v].append(x)
    for sc in res:
        print(sc)
        for v, xs in res[sc].items():
            tot = [x["solo"]["total"] for x in xs]
            parts = {k: round(sum(x["solo"].get(k, 0) for x in xs) / len(xs), 2)
                     for k in ("primary", "extend", "shadow", "shade", "tiles") if any(k in x["solo"] for x in xs)}
            pipe = [x["pipe_fps"] for x in xs if x.get("pipe_fps")]
            print(f"   {v:9s} solo best {min(tot):9.3f} mean {sum(tot) / len(tot):9.3f} {parts}"
                  + (f" pipe {pipe}" if pipe else ""))


if __name__ == "__main__":
    main()
