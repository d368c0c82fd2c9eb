#!/bin/bash
# Counter exploration: list counters, then one PMC pass per argument (a comma-free, space-separated
# counter set in quotes) over one sample-mode C3 frame (SPP, default 64; MODE=compat for compat).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1; echo "list rc=$?"
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/one_frame.py c3 ${SPP:-64} ${MODE:-sample} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; tail -1 $OUT/p$i.log | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
