#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
#   tools/gpu_steps.sh "name|seconds|command" ...
# A step that fails normally (exit 1: a failed test or check) lets the next one run; a step that
# times out, aborts, crashes or faults ends the sequence (nothing more touches the GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
status=0
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "== $name ($secs s): $cmd"
    mkdir -p "$(dirname "gpurun_out/$name.log")"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc"
    tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then
        status=$rc
        if [ $rc -ne 1 ]; then echo "== stopping after $name (rc $rc)"; exit $rc; fi
    fi
done
exit $status
