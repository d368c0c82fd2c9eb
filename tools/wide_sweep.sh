#!/bin/bash
# Wide-tree build parameter sweep (GPU): C3 @64 spp, C5 @16, C2 @256, sample mode.
for leaf in 1 2 3; do
  for trav in 0.5 1 2; do
    for cfg in "c3 64" "c5 16" "c2 256"; do
      r=$(PT_WIDE_MAX_LEAF=$leaf PT_WIDE_TRAV_COST=$trav timeout -k 5 100 python tools/wide_vs_ref.py $cfg 2>&1 | grep "^wide")
      echo "leaf $leaf trav $trav $cfg: $r"
    done
  done
done
