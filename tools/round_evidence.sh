#!/bin/bash
# One GPU call that regenerates the round's evidence (run on the GPU box from the
# repo root): parity tests, rocprof kernel-trace + PMC summaries per workload,
# then bench lines that quote those summaries. Everything lands in gpurun_out/.
#   tools/round_evidence.sh r1
tag=${1:-r1}
S=tools/gpu_steps.sh
mkdir -p gpurun_out/ev
$S 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ::: \
   900 tools/profile_round.sh $tag ::: \
   900 tools/profile_round.sh ${tag}_01 01 ::: \
   900 tools/profile_round.sh ${tag}_02 02 ::: \
   900 tools/profile_round.sh ${tag}_03 03 ::: \
   900 tools/profile_round.sh ${tag}_c5 c5 "--spp 64" || exit $?
# the bench lines below price their roofline with these (bench.py newest_profile)
cp gpurun_out/prof_$tag/${tag}_pmc.json profiles/${tag}_pmc.json
for w in 01 02 03; do cp gpurun_out/prof_${tag}_$w/${tag}_${w}_pmc.json profiles/${tag}_pmc_$w.json; done
cp gpurun_out/prof_${tag}_c5/${tag}_c5_pmc.json profiles/${tag}_pmc_c5.json
for wl in 04vs 01 02 03 c5; do
    $S 600 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
done
$S 200 python bench.py --serial --no-cpu-baseline > gpurun_out/ev/bench_04vs_serial.json
$S 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log
