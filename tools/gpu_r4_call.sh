#!/bin/bash
# Round-4 GPU call: full-frame parity of the lazy ray origin, then its A/B on
# the k_tiles scenes (pipelined) against the previous commit (head tree).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4v_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_run.py --rounds 3 --frames 40 main head -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab25.txt 2>&1
