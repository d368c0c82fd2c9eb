#!/bin/bash
# Leaf splitting on/off (the wide tree is built once per process): C3 / C2 / C5, sample mode.
for cfg in "c3 256" "c2 1024" "c5 64"; do
  for sp in 1 0; do
    r=$(PT_WIDE_SPLIT_LEAVES=$sp REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg sample 2>&1 | tail -1)
    echo "split $sp $cfg: $r"
  done
done
