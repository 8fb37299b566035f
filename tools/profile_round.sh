#!/usr/bin/env bash
# Kernel-trace stats + separate PMC passes of a bench workload (one counter
# group per run, MI355X_MICROARCH.md §rocprofv3 PMC slots), then per-kernel
# summaries. Run on the GPU box from the repo root:
#   tools/profile_round.sh <tag> [workload] [extra bench args]
#   tools/profile_round.sh r1                 # 04vs, the headline config
#   tools/profile_round.sh r1_c5 c5 "--spp 64" # C5 (same per-launch sizes: 32-spp chunks)
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/.
set -euo pipefail
tag=${1:-r1}
wl=${2:-04vs}
extra=${3:-}
out=gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null

if [ "$wl" == "c5" ]; then steps="--steps 2 --warmup 1"; psteps="--steps 1 --warmup 1"; else steps="--steps 10 --warmup 2"; psteps="--steps 3 --warmup 1"; fi
# LDS-tile workloads (04vs, 01): frames overlap in the pipelined bench, and
# every frame that overlaps a pending one runs k_tiles<false, true> (whole-
# tile units); a frame alone runs k_tiles<false, false> (sample-group
# slices). The counter passes run the pipelined bench, so the summary holds
# a per-launch count for both variants (the profiler serialises dispatches,
# so each count is the launch's own); bench.py prices the timed region's
# launches with them. A second kernel trace runs the frames serially (one
# launch on the chip at a time): the solo launches of the roofline's
# secondary figure.
ser=""
if [ "$wl" == "04vs" ] || [ "$wl" == "01" ]; then ser="--serial"; fi
if [ "$wl" == "c5" ]; then psteps="--steps 1 --warmup 1"; else psteps="--steps 6 --warmup 1"; fi
B="bench.py --workload $wl $psteps --no-cpu-baseline --no-profile $extra"

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
    -- python3 bench.py --workload $wl $steps --no-cpu-baseline $extra > "$out/trace_bench.json"
echo "trace done"
if [ -n "$ser" ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_serial" -o run \
        -- python3 bench.py --workload $wl $steps --no-cpu-baseline --serial $extra > "$out/trace_serial_bench.json"
    echo "serial trace done"
fi
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 $B > /dev/null
echo "fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 $B > /dev/null
echo "write done"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$out/sq1" -o run -- python3 $B > /dev/null
echo "sq1 done"
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR \
    SQ_THREAD_CYCLES_VALU TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$out/sq2" -o run -- python3 $B > /dev/null
echo "sq2 done"
python3 tools/pmc_summary.py stats "$out/trace" > "$out/${tag}_kernel_stats.md"
if [ -n "$ser" ]; then
    python3 tools/pmc_summary.py stats "$out/trace_serial" > "$out/${tag}_serial_kernel_stats.md"
fi
python3 tools/pmc_summary.py traffic --fetch "$out/fetch" --write "$out/write" --sq "$out/sq1" --sq "$out/sq2" \
    -o "$out/${tag}_pmc.json"
