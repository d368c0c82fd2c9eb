#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 600 python tools/wave_times2.py > gpurun_out/wt3.log 2>&1
rc=$?; echo "wt rc=$rc"; grep '^{' gpurun_out/wt3.log | cut -c1-330
exit $rc
