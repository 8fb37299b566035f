#!/bin/bash
# Round-4 GPU call: GPU tests of the tree; the secondary-ray sort variant
# (RR_RAY_SORT=1) through the split-path parity tests; the split-path A/B
# (trace block size, LDS top depth, next-node touch, ray sort, box margins);
# the k_tiles uniform-kz A/B; the counter calibration probe. Stops at the
# first failing step.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || exit $rc
RR_LIB_PATH=$PWD/diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd/build/ab_sort/librr.so \
timeout -k 10 300 python -u -m pytest tests/test_gpu_physics.py -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "full_frame or bench_config or stack_drops or reduced" > gpurun_out/r4_sort_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_sort_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python tools/ab_run.py --rounds 2 main pf sort b256 t128 s8t768 pernode r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab4.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_run.py --rounds 3 --frames 40 main nokz r3 -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab5.txt 2>&1 || exit $?
bash tools/gpu_fetch_probe.sh > gpurun_out/fetch_probe.log 2>&1
