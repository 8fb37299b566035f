#!/usr/bin/env bash
# PC sampling of one bench workload (rocprofv3, host-trap method): where the
# waves of the hot kernel spend their time, per instruction. Run on the GPU box
# from the repo root:
#   tools/pc_sample.sh <tag> [workload] [extra bench args]
# Output under gpurun_out/pcs_<tag>/ (CSV); tools/pc_summary.py aggregates it.
set -euo pipefail
tag=${1:-r3}
wl=${2:-04vs}
extra=${3:-}
out=gpurun_out/pcs_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
    --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d "$out" -o run \
    -- python3 bench.py --workload $wl --serial --steps 6 --warmup 1 --no-cpu-baseline --no-profile $extra \
    > "$out/bench.json"
echo "pc sampling done"
