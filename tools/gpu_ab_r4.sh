#!/bin/bash
# Round-4 A/B call on the GPU box: trace-block size / LDS top depth / box
# margin variants on the split-path scenes. Variants: tools/ab_variants.sh
# builds (build/ab_<name>).
mkdir -p gpurun_out
timeout -k 10 1050 python tools/ab_run.py --rounds 2 main pf b256 t128 s8t768 pernode r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab4.txt 2>&1
