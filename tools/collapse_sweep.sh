#!/bin/bash
# Wide-tree collapse A/B (GPU): greedy vs cost-optimal with several primitive-test weights.
run() {
  for cfg in "c3 256" "c5 64" "c2 1024"; do
    r=$(env "$@" REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg sample | tail -1)
    echo "$* $cfg: $r"
  done
}
run PT_WIDE_COLLAPSE=greedy
for pc in 0.5 1 1.5 2.5; do run PT_WIDE_PRIM_COST=$pc; done
