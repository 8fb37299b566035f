#!/bin/bash
# Round-4 GPU call: split-path A/B isolating the costs of the watertight test
# (timing-only builds: no axis permutation, no exact fallback) and the
# per-node box margin, against main and round 3.
mkdir -p gpurun_out
timeout -k 10 480 python tools/ab_run.py --rounds 2 main norot noexact pn r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab8.txt 2>&1
