#!/bin/bash
# Round-4 GPU call: split-path shading kernels at 5 / 6 waves per SIMD against
# the compiler's 4.
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_run.py --rounds 2 main sw5 sw6 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab24.txt 2>&1
