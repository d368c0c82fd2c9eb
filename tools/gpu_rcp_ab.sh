#!/bin/bash
# Exhaustive reciprocal check, then the fast-reciprocal build vs the IEEE-division build (GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=path-tracer-cuda-opengl_amd
timeout -k 10 120 ./tools/micro/rcp_check || exit $?
for cfg in "c3 256" "c5 64" "c2 1024"; do
  timeout -k 10 600 bash tools/libs_ab.sh "$cfg" 2 ieee=$L/variants/libpt_ieee.so rcp=$L/libpt.so || exit $?
done
MODE=compat timeout -k 10 600 bash tools/libs_ab.sh "c3 64" 2 ieee=$L/variants/libpt_ieee.so rcp=$L/libpt.so || exit $?
