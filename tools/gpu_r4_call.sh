#!/bin/bash
# Round-4 GPU call: GPU tests; the shadow-packet variant through the split-path
# parity tests; the split-path A/B: pixel-major path index (main), + bounce-0
# shadow packets (shpk), pixel packets over the sample-major index (pkall tree),
# round 3.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4m_tests.log
[ $rc -eq 0 ] || exit $rc
RR_LIB_PATH=$PWD/diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd/build/ab_shpk/librr.so \
timeout -k 10 300 python -u -m pytest tests/test_gpu_physics.py -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "full_frame or bench_config or stack_drops or reduced" > gpurun_out/r4_shpk_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_shpk_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python tools/ab_run.py --rounds 2 main shpk pkall r3 -- scenes/02_physics-standin.rrscene:90:64 scenes/03_physics-2-standin.rrscene:300:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab15.txt 2>&1
