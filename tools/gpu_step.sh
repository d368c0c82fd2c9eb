#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faults,
# aborts or times out (exit codes other than 0 / 1).  Usage: gpu_step.sh OUTDIR "secs:cmd" ...
out=$1; shift
mkdir -p "$out"
i=0
for step in "$@"; do
    i=$((i + 1))
    secs=${step%%:*}
    cmd=${step#*:}
    echo "[step $i] $cmd" | tee -a "$out/steps.log"
    timeout -k 10 "$secs" bash -c "$cmd" > "$out/step$i.log" 2>&1
    rc=$?
    echo "[step $i] rc=$rc" | tee -a "$out/steps.log"
    tail -3 "$out/step$i.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
