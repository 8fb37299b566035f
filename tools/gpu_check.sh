#!/bin/bash
# One GPU call for the edit -> measure loop (run on the GPU box from the repo
# root): the -m gpu tests, then the default bench line, each under its own
# time limit, logs under gpurun_out/. A timeout / abort / crash of a step ends
# the call (nothing else touches a possibly faulted GPU).
#   tools/gpu_check.sh <tag> [extra pytest args, e.g. -k expr]
set -u
tag=${1:-chk}
shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc: $(grep -E '^(=+ )?[0-9]+ (passed|failed)' gpurun_out/${tag}_tests.log | tail -1)"
grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head -5
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc2=$?
echo "bench rc=$rc2"
python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/${tag}_bench.json') if l.startswith('{')][-1])
r=d.get('roofline') or {}
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', {k: r.get(k) for k in ('avg_launch_ms','frac','valu_per_launch')}, 'solo', (r.get('solo') or {}).get('avg_launch_ms'))
" || true
exit $(( rc2 >= 124 ? rc2 : 0 ))
