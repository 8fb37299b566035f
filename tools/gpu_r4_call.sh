#!/bin/bash
# Round-4 GPU call: split-path re-tune on the pixel-major order: lane-refill
# threshold 44 / 58 (main 52) and 7 waves per SIMD for the trace kernels.
mkdir -p gpurun_out
timeout -k 10 480 python tools/ab_run.py --rounds 2 main rf44 rf58 w7 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab20.txt 2>&1
