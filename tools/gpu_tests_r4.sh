#!/bin/bash
# Round-4 GPU tests, the k_tiles uniform-kz A/B and the counter calibration probe.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_run.py --rounds 3 --frames 40 main nokz r3 -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab5.txt 2>&1 || exit $?
bash tools/gpu_fetch_probe.sh > gpurun_out/fetch_probe.log 2>&1
