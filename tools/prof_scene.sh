#!/bin/bash
# Kernel-trace stats + two SQ/TCC counter passes of one diag_traversal.py frame.
#   TAG=x SCENE=scenes/... FRAME=90 SPP=16 tools/prof_scene.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
O=gpurun_out/prof_${TAG:-scene}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/diag_traversal.py ${SCENE:-scenes/02_physics-standin.rrscene} ${FRAME:-90} ${SPP:-16} > $O/diag.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 tools/diag_traversal.py ${SCENE:-scenes/02_physics-standin.rrscene} ${FRAME:-90} ${SPP:-16} > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/sq2 -o run -- python3 tools/diag_traversal.py ${SCENE:-scenes/02_physics-standin.rrscene} ${FRAME:-90} ${SPP:-16} > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/diag_traversal.py ${SCENE:-scenes/02_physics-standin.rrscene} ${FRAME:-90} ${SPP:-16} > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/diag_traversal.py ${SCENE:-scenes/02_physics-standin.rrscene} ${FRAME:-90} ${SPP:-16} > /dev/null
python3 tools/pmc_summary.py stats $O/trace > $O/stats.md
python3 tools/pmc_summary.py traffic --fetch $O/fetch --write $O/write --sq $O/sq1 --sq $O/sq2 -o $O/pmc.json
