#!/bin/bash
# Round-4 GPU call: split-path A/B bisecting the round-4 cost against round 3
# (timing-only builds: mt = round 3's triangle test; allr3 = mt + no box margin
# + no used-slot mask + no stack-drop counter; nodrop = no drop counter).
mkdir -p gpurun_out
timeout -k 10 480 python tools/ab_run.py --rounds 2 main mt allr3 nodrop r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab12.txt 2>&1
