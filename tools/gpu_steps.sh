#!/bin/bash
# Runs GPU steps in sequence on the gpurun box, each under its own time limit.
# A step that ends in a plain failure (exit 1-123, e.g. failing tests) lets the
# next step run; a timeout (124/137), abort (134), segfault (139) or any other
# signal ends the whole call so nothing else touches a possibly-faulted GPU.
#   tools/gpu_steps.sh <seconds> <cmd...> ::: <seconds> <cmd...> ::: ...
set -u
mkdir -p gpurun_out
step=()
run_step() {
    local secs=$1; shift
    echo "=== [$(date +%T)] step (${secs}s): $*" >&2
    timeout -k 10 "$secs" "$@"
    local rc=$?
    echo "=== step rc=$rc" >&2
    if [ $rc -ge 124 ]; then
        echo "=== stopping: step ended with rc=$rc" >&2
        exit $rc
    fi
}
for a in "$@"; do
    if [ "$a" == ":::" ]; then
        run_step "${step[@]}"
        step=()
    else
        step+=("$a")
    fi
done
if [ ${#step[@]} -gt 0 ]; then run_step "${step[@]}"; fi
exit 0
