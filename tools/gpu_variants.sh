#!/bin/bash
# A/B of library builds: one C3 frame per (variant, mode, leaf batch).  VARIANTS = names under
# variants/ ("base" = libpt.so); LEAFS = PT_LEAF_BATCH values.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do for m in ${MODES:-compat}; do for lb in ${LEAFS:-0}; do for sb in ${SHADES:-0}; do
  lib=""; [ "$v" != base ] && lib=path-tracer-cuda-opengl_amd/variants/libpt_$v.so
  PT_LIB=$lib PT_ITER_STATS=1 PT_LEAF_BATCH=$lb PT_SHADE_BATCH=$sb timeout -k 10 120 python tools/one_frame.py ${CFG:-c3} ${SPP:-1024} $m > gpurun_out/var.log 2>&1; rc=$?
  echo "$v $m L$lb S$sb: $(grep '^\[pt\]' gpurun_out/var.log | tail -3 | cut -c6- | tr '\n' ' ') $(grep '^{' gpurun_out/var.log | cut -c28-60)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/var.log; exit $rc; fi
done; done; done; done
