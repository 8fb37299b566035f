#!/bin/bash
# Round-4 GPU call: k_tiles at 5 / 6 waves per SIMD against main's 4 (04vs /
# 01, pipelined frames), two more rounds.
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_run.py --rounds 3 --frames 40 main tw5 tw6 -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab22.txt 2>&1
