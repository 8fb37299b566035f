#!/bin/bash
# One PMC pass (instruction mix + cycles) of the k_tiles frame for each A/B
# variant (tools/ab_variants.sh builds), on the GPU box from the repo root:
#   tools/pmc_variants.sh <frame> <variant>...
# Prints per variant the counters of the timed k_tiles launch (tools/pmc_summary.py).
set -eu
frame=$1; shift
PKG=diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd
mkdir -p gpurun_out/pmcv
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "$@"; do
    d=gpurun_out/pmcv/$v
    RR_LIB_PATH=$PWD/ab_builds/$v/librr.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
        --output-format csv -d $d -o run -- python3 tools/render_once.py $frame > /dev/null
    python3 - "$d" "$v" <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_tiles<false>" in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
last = sorted(acc, key=int)[-1]
c = {k: sum(x) for k, x in acc[last].items()}
print(v, {k: round(x / 1e6, 2) for k, x in sorted(c.items())}, "(millions)")
PY
done
