#!/bin/bash
# Iteration session: GPU tests, short bench, optional sweep.  Time-limited steps; stop on crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1200 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$SWEEP" ]; then
timeout -k 10 900 python tools/sweep.py ${SWEEP_CFG:-c3} ${SPP:-128} ${SETTINGS} > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep '^{' gpurun_out/sweep.log | cut -c1-160
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log
exit $rc
