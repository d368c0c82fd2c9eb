#!/bin/bash
# One GPU-box session for an experiment: GPU tests, then A/B of library builds (LIBS, via
# tools/libs_ab.sh) and of run-time settings on rank shares (PART_V, via tools/part_ab.py).
# Every GPU step has its own time limit and the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$LIBS" ]; then
  IFS=';' read -ra CFGS <<< "${AB_CFGS:-c3 256}"
  for c in "${CFGS[@]}"; do
    bash tools/libs_ab.sh "$c" ${AB_ROUNDS:-3} $LIBS > gpurun_out/libs_ab.log 2>&1 || { cat gpurun_out/libs_ab.log; exit 1; }
    cat gpurun_out/libs_ab.log
  done
fi
if [ -n "$PART_V" ]; then
  for n in ${PART_N:-8 1}; do
    timeout -k 10 300 python tools/part_ab.py $n ${PART_SPP:-1024} ${PART_ROUNDS:-3} $PART_V > gpurun_out/part_ab_$n.log 2>&1 || { cat gpurun_out/part_ab_$n.log; exit 1; }
    cat gpurun_out/part_ab_$n.log
  done
fi
echo session-ok
