#!/bin/bash
# Round-4 final check of the tree on the GPU box: the -m gpu suite, smoke()
# and the default bench line.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_final_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_final_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err
