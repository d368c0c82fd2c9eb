#!/bin/bash
# PLOC radius / traversal-cost sweep for the device-built wide tree (GPU): frame ms on C2/C3/C5.
for r in 8 16 32 64; do
  for t in 0.5 1 2; do
    echo "radius $r trav $t"
    PT_PLOC_RADIUS=$r PT_WIDE_TRAV_COST=$t timeout -k 5 200 python tools/wide_build_ab.py c3 c5 2>&1 | grep " device "
  done
done
