#!/bin/bash
# Copies the summaries of tools/round_evidence.sh calls (merged back into
# gpurun_out/) into profiles/ (tracked). Run here, after the GPU call(s):
#   tools/collect_evidence.sh r3
# Workloads whose outputs are missing are skipped (and listed).
set -uo pipefail
tag=${1:-r1}
for p in "" _01 _02 _03 _c5; do
    d=gpurun_out/prof_${tag}${p}
    if [ ! -f $d/${tag}${p}_kernel_stats.md ]; then echo "skip profile ${tag}${p}"; continue; fi
    cp $d/${tag}${p}_kernel_stats.md profiles/${tag}${p}_kernel_stats.md
    cp $d/trace/run_kernel_stats.csv profiles/${tag}${p}_kernel_stats.csv
    cp $d/${tag}${p}_pmc.json profiles/${tag}_pmc${p}.json
    grep '^{' $d/trace_bench.json > profiles/${tag}${p}_bench_under_rocprof.json
    if [ -f $d/${tag}${p}_serial_kernel_stats.md ]; then
        cp $d/${tag}${p}_serial_kernel_stats.md profiles/${tag}${p}_serial_kernel_stats.md
        cp $d/trace_serial/run_kernel_stats.csv profiles/${tag}${p}_serial_kernel_stats.csv
        grep '^{' $d/trace_serial_bench.json > profiles/${tag}${p}_serial_bench_under_rocprof.json
    fi
done
for wl in 04vs 01 02 03 c5 04vs_serial 04vs_driver_config; do
    f=gpurun_out/ev/bench_$wl.json
    if [ -f $f ] && grep -q '^{' $f; then grep '^{' $f > profiles/${tag}_bench_$wl.json; else echo "skip bench $wl"; fi
done
if [ -f gpurun_out/ev/smoke.log ]; then grep -v '^===' gpurun_out/ev/smoke.log > profiles/${tag}_smoke.log; fi
if [ -f gpurun_out/ev_log.txt ]; then grep -E '[0-9]+ passed' gpurun_out/ev_log.txt | head -1 > profiles/${tag}_gpu_tests_summary.txt; fi
