#!/bin/bash
# Interleaved comparison of several library builds (GPU): libs_ab.sh "c3 256" rounds name=lib.so ...
cfg=$1; rounds=$2; shift 2
for r in $(seq $rounds); do
  for v in "$@"; do
    name=${v%%=*}; lib=${v#*=}
    out=$(PT_LIB=$lib REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg ${MODE:-sample} | tail -1)
    echo "$name $cfg $out"
  done
done
