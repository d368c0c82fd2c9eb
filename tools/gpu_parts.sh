#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${NS:-2 4 8}; do for m in ${MODES:-sample compat}; do
timeout -k 10 300 python tools/part_time.py $n $m > gpurun_out/parts_${n}_$m.log 2>&1; rc=$?
cat gpurun_out/parts_${n}_$m.log | grep '^{'; if [ $rc -ne 0 ]; then tail -5 gpurun_out/parts_${n}_$m.log; exit $rc; fi
done; done
