#!/bin/bash
# GPU tests + scheduler sweep (c3, c2) + SQ counters per kernel.  Each GPU step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1200 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python tools/sweep.py c3 ${SPP:-128} ${SETTINGS} > gpurun_out/sweep_c3.log 2>&1
rc=$?; echo "sweep c3 rc=$rc"; grep '^{' gpurun_out/sweep_c3.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/sweep.py c2 ${SPP2:-256} ${SETTINGS} > gpurun_out/sweep_c2.log 2>&1
rc=$?; echo "sweep c2 rc=$rc"; grep '^{' gpurun_out/sweep_c2.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PMC" ]; then
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d gpurun_out/pmc_sweep -o run --output-format csv -- python3 tools/sweep.py c3 64 ${PMC_SETTINGS} > gpurun_out/pmc_sweep.log 2>&1
rc=$?; echo "pmc rc=$rc"
fi
exit $rc
