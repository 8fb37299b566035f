#!/bin/bash
# Round-4 GPU call: GPU tests, then k_tiles per-variant occupancy (main: whole
# tiles at 5 waves, slices at 4) against both at 5 (tw5).
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4t_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_run.py --rounds 3 --frames 40 main tw5 -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab23.txt 2>&1
