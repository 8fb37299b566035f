#!/bin/bash
# Round-4 GPU tests + counter calibration probe.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_fetch_probe.sh > gpurun_out/fetch_probe.log 2>&1
