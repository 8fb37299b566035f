#!/bin/bash
# Round-4 GPU call: the guarded-reciprocal shading variant (srcp) through the
# full-frame parity tests, then its A/B against main on the k_tiles scenes
# (pipelined) and two split-path scenes.
mkdir -p gpurun_out
RR_LIB_PATH=$PWD/diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd/build/ab_srcp/librr.so \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "full_frame_bit_exact or furnace or point_light" > gpurun_out/r4_srcp_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_srcp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_run.py --rounds 3 --frames 40 main srcp -- scenes/04_very-simple-standin.rrscene:5:128 scenes/01_simple-animation.rrscene:20:128 > gpurun_out/ab18.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab_run.py --rounds 2 main srcp -- scenes/02_physics-standin.rrscene:90:64 scenes/c5_synthetic-10m.rrscene:150:16 > gpurun_out/ab19.txt 2>&1
