#!/bin/bash
# Queue a gpurun call: retry only while the pool has no box free (gpurun exit 3, nothing ran,
# nothing charged), up to ~40 minutes.  Any other outcome -- including a failed GPU step -- is final.
#   tools/gpurun_wait.sh <timeout-seconds> <log> <command>
lim=$1; log=$2; shift 2
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$log" 2>&1
    rc=$?
    if [ $rc -ne 3 ] && ! grep -q "no free box right now\|backing off\|all .* GPU slot(s) on this pod are busy" "$log"; then exit $rc; fi
    sleep 120
done
exit 3
