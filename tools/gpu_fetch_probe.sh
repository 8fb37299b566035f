#!/bin/bash
# PMC byte-counter calibration on the GPU box (tools/fetch_probe.hip): one
# rocprofv3 pass per counter group, then the ratios (tools/fetch_probe.py).
set -u
out=gpurun_out/fetch_probe
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- tools/bin/fetch_probe \
    > $out/known.json || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum \
    --output-format csv -d $out/req -o run -- tools/bin/fetch_probe > /dev/null || exit $?
python3 tools/fetch_probe.py $out/known.json $out/fetch $out/req > $out/fetch_probe.json
cat $out/fetch_probe.json
