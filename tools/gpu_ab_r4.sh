mkdir -p gpurun_out
timeout -k 10 700 python tools/ab_run.py --rounds 2 main pernode w7 r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab4.txt 2>&1 || exit $?
timeout -k 10 400 python tools/ab_run.py --rounds 3 --frames 40 main nokz r3 -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab5.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
tail -3 gpurun_out/r4c_tests.log
