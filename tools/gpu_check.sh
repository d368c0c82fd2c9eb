#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench.  Every GPU step has its own time
# limit; a crash/abort/timeout (rc not in {0,1}) ends the script without further GPU work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SPP=${SPP:-64}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_short.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_short.log
exit $rc
