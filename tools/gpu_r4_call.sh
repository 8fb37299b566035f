#!/bin/bash
# Round-4 GPU call: GPU tests, then the split-path A/B of the stored-exponent
# margin (main) against the previous commit (head tree) and round 3.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4o_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_run.py --rounds 2 main head r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab17.txt 2>&1
