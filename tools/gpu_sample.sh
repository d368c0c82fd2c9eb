#!/bin/bash
# Sample-mode session: its GPU tests, then bench in compat and sample mode at several chunk sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -k "${PYTEST_K:-sample}" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in ${CHUNKS:-16 64 256}; do
timeout -k 10 300 python bench.py --rng sample --chunk $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s$c.log 2>&1
rc=$?; echo "chunk $c rc=$rc"; grep '^{' gpurun_out/bench_s$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
if [ $rc -ne 0 ]; then exit $rc; fi
done
