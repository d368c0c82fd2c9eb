#!/bin/bash
# Sample-mode session: its GPU tests, then bench in sample mode for several PT_UNIT_SPLIT values.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -k "${PYTEST_K:-sample}" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for sp in ${SPLITS:-4}; do
PT_UNIT_SPLIT=$sp timeout -k 10 300 python bench.py --rng sample --steps 2 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_u$sp.log 2>&1
rc=$?; echo "split $sp rc=$rc"; grep '^{' gpurun_out/bench_u$sp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
if [ $rc -ne 0 ]; then exit $rc; fi
done
