#!/bin/bash
# Wavefront thresholds for the wide kernel (GPU): C3 @64 spp sample mode, 2 frames each.
for lb in 16 24 32 40; do
  for sb in 24 32 40; do
    r=$(PT_LEAF_BATCH=$lb PT_SHADE_BATCH=$sb REPEAT=3 timeout -k 5 100 python tools/one_frame.py c3 64 sample 2>&1 | tail -1)
    echo "leaf $lb shade $sb: $r"
  done
done
