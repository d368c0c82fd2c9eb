#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/wave_times2.py > gpurun_out/wt2.log 2>&1
rc=$?; echo "wt rc=$rc"; cat gpurun_out/wt2.log | grep '^{'
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-300
exit $rc
