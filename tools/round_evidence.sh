#!/bin/bash
# Regenerates the round's evidence on the GPU box (from the repo root), in two
# parts that each fit one gpurun call: parity tests, rocprof kernel-trace + PMC
# summaries per workload, then bench lines that quote those summaries.
# Everything lands in gpurun_out/; tools/collect_evidence.sh copies it.
#   tools/round_evidence.sh r3 a   # -m gpu tests, smoke, 04vs (+ serial), 01, 02
#   tools/round_evidence.sh r3 b   # 03, c5
#   tools/round_evidence.sh r3 c   # the split-path workloads 02, 03, c5 again
# Smaller parts, one gpurun call each (round 6):
#   t  -m gpu tests + smoke;  k  04vs (+ serial), 01;  s  02, 03;  5  c5
tag=${1:-r1}
part=${2:-a}
S=tools/gpu_steps.sh
mkdir -p gpurun_out/ev
prof() {  # workload key ("" for 04vs), profile_round args
    local k=$1; shift
    $S 600 tools/profile_round.sh "$@" || exit $?
    local d=gpurun_out/prof_${tag}${k:+_$k}
    cp $d/${tag}${k:+_$k}_pmc.json profiles/${tag}_pmc${k:+_$k}.json  # bench.py prices its roofline with it
}
if [ "$part" == "t" ]; then
    $S 500 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit $?
    $S 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log || exit $?
elif [ "$part" == "k" ]; then
    prof "" $tag
    prof 01 ${tag}_01 01
    for wl in 04vs 01; do
        $S 300 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
    done
    $S 200 python bench.py --serial --no-cpu-baseline > gpurun_out/ev/bench_04vs_serial.json || exit $?
    $S 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ev/bench_04vs_driver_config.json || exit $?
elif [ "$part" == "s" ]; then
    prof 02 ${tag}_02 02
    prof 03 ${tag}_03 03
    for wl in 02 03; do
        $S 400 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
    done
elif [ "$part" == "5" ]; then
    prof c5 ${tag}_c5 c5 "--spp 64"
    $S 400 python bench.py --workload c5 > gpurun_out/ev/bench_c5.json || exit $?
elif [ "$part" == "a" ]; then
    $S 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
    $S 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log || exit $?
    prof "" $tag
    prof 01 ${tag}_01 01
    prof 02 ${tag}_02 02
    for wl in 04vs 01 02; do
        $S 300 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
    done
    $S 200 python bench.py --serial --no-cpu-baseline > gpurun_out/ev/bench_04vs_serial.json || exit $?
elif [ "$part" == "c" ]; then
    prof 02 ${tag}_02 02
    prof 03 ${tag}_03 03
    prof c5 ${tag}_c5 c5 "--spp 64"
    for wl in 02 03 c5; do
        $S 400 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
    done
else
    prof 03 ${tag}_03 03
    prof c5 ${tag}_c5 c5 "--spp 64"
    for wl in 03 c5; do
        $S 400 python bench.py --workload $wl > gpurun_out/ev/bench_$wl.json || exit $?
    done
fi
