#!/bin/bash
# Interleaved A/B of two library builds (GPU), one process per run: lib_ab.sh OLD.so NEW.so "c3 256" [rounds]
# (pass "compat" as a 5th argument for compat mode)
old=$1; new=$2; cfg=$3; rounds=${4:-3}; mode=${5:-sample}
for r in $(seq $rounds); do
  for v in old new; do
    lib=$old; [ $v = new ] && lib=$new
    out=$(PT_LIB=$lib REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg $mode | tail -1)
    echo "$v $cfg $out"
  done
done
