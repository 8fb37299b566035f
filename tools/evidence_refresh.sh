#!/bin/bash
# Re-profiles and re-benches a subset of workloads on the GPU box (repo root),
# the same steps as tools/round_evidence.sh for those workloads only:
#   tools/evidence_refresh.sh <tag> <workload>...     e.g.  r2 04vs 01 c5
# Copies the PMC summaries into profiles/ (the bench lines price their roofline
# with them) and leaves the bench lines in gpurun_out/ev/bench_<wl>.json.
tag=$1; shift
S=tools/gpu_steps.sh
mkdir -p gpurun_out/ev
for wl in "$@"; do
    if [ "$wl" == "04vs" ]; then t=$tag; else t=${tag}_$wl; fi
    extra=""; [ "$wl" == "c5" ] && extra="--spp 64"
    $S 400 tools/profile_round.sh $t $wl "$extra" || exit $?
    if [ "$wl" == "04vs" ]; then cp gpurun_out/prof_$t/${t}_pmc.json profiles/${tag}_pmc.json
    else cp gpurun_out/prof_$t/${t}_pmc.json profiles/${tag}_pmc_$wl.json; fi
done
for wl in "$@"; do
    $S 300 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
done
