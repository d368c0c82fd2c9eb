#!/bin/bash
# A/B of library variants on one rank's share of the C3 frame: VARIANTS (base = libpt.so), PARTS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base}; do for n in ${PARTS:-1 8}; do
  lib=""; [ "$v" != base ] && lib=path-tracer-cuda-opengl_amd/variants/libpt_$v.so
  echo "$v: $(PT_LIB=$lib timeout -k 10 200 python tools/part_time.py $n sample 1024 | tr "\n" " ")" || exit 1
done; done
