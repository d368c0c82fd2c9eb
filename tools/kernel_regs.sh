#!/bin/bash
# Per-kernel VGPRs / spills / occupancy of a pt_device.hip source (default: the working tree's),
# compiled with the package's flags:  tools/kernel_regs.sh [file.hip] [grep-pattern]
f=${1:-path-tracer-cuda-opengl_amd/csrc/pt_device.hip}; pat=${2:-renderKernelWF}
cd "$(dirname "$0")/.." || exit 2
P=path-tracer-cuda-opengl_amd
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -fno-fast-math -Iinclude -I$P/host -I$P/csrc -Wall \
  --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -mllvm --enable-post-misched=0 $EXTRA \
  -c "$f" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$pat" '/Function Name:/ {name=$(NF-1); show=(name ~ pat)} show && /VGPRs:|VGPRs Spill:|Occupancy/ {sub(/.*remark: +/, ""); sub(/ \[-Rpass.*/, ""); printf "%s  %s\n", name, $0}' |
  c++filt | sed 's/(anonymous namespace):://'
