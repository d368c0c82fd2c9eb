#!/bin/bash
# Wide-tree build parameter sweep (GPU, one process per setting: the tree is built once per
# scene): C3 @256 spp and C5 @64 spp, sample mode, fastest of 3 frames.
for leaf in 1 2 3; do
  for trav in 0.5 1 1.5; do
    for cfg in "c3 256" "c5 64"; do
      r=$(PT_WIDE_MAX_LEAF=$leaf PT_WIDE_TRAV_COST=$trav REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg sample 2>&1 | tail -1)
      echo "leaf $leaf trav $trav $cfg: $r"
    done
  done
done
