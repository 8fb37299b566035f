#!/usr/bin/env python3
"""Register / scratch / occupancy table of the device kernels, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (one translation unit per call).

    python tools/res_usage.py wavefront.hip [tiles.hip ...] [--extra '-DFOO=1']

Compiles each file device-only with the Makefile's device flags into /tmp and
prints one line per kernel: VGPRs, AGPRs, VGPR spills, SGPR spills, scratch
bytes per lane and waves per SIMD. Build-time inspection only."""
import argparse
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                    "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd", "csrc")
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
TU_FLAGS = {"tiles.hip": os.environ.get("RR_TILES_TUFLAGS", "-fno-slp-vectorize").split()}


def usage(src, extra):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"),
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-Xclang", "-target-feature", "-Xclang",
           "-packed-fp32-ops", "--cuda-device-only", "-c", src, "-o", "/tmp/res_usage.o",
           "-Rpass-analysis=kernel-resource-usage"] + TU_FLAGS.get(os.path.basename(src), []) + extra
    p = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
    if p.returncode:
        sys.stderr.write(p.stderr)
        raise SystemExit(p.returncode)
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|"
                      r"Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    return rows


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(I[^E]*E)?", name)
    if not m:
        return name[:40]
    tmpl = re.findall(r"Lb([01])E", m.group(2) or "")
    return m.group(1) + ("<" + ",".join(tmpl) + ">" if tmpl else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    print(f"{'kernel':34s} {'VGPR':>5s} {'AGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'scratch':>7s} {'waves':>5s}")
    for f in a.files:
        for r in usage(f, a.extra.split()):
            if not r["name"].startswith("_Z") or "k_" not in r["name"]:
                continue
            print(f"{short(r['name']):34s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} "
                  f"{r.get('VGPRs Spill', '?'):>6s} {r.get('SGPRs Spill', '?'):>6s} "
                  f"{r.get('ScratchSize [bytes/lane]', '?'):>7s} {r.get('Occupancy [waves/SIMD]', '?'):>5s}")


if __name__ == "__main__":
    main()
