#!/bin/bash
# FETCH_SIZE calibration on the GPU box (run via gpurun): tools/micro/fetch_calib under separate
# rocprofv3 --pmc passes, one per counter group and access mode -> gpurun_out/fetch_calib/.
# tools/fetch_calib.py then turns the CSVs into profiles/fetch_calib.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/fetch_calib
mkdir -p $OUT
timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for mode in ${MODES:-stream g128 g64s128 g80s128 g80 g80mall g80warm g48}; do
    timeout -k 10 60 tools/micro/fetch_calib $mode > $OUT/$mode.json 2> $OUT/$mode.err || exit $?
    for pass in "fetch:FETCH_SIZE" "ea:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "hit:TCC_HIT_sum TCC_MISS_sum" \
                "bub:TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum"; do
        name=${pass%%:*}; ctrs=${pass#*:}
        timeout -s KILL 60 rocprofv3 --pmc $ctrs -d $OUT/${mode}_$name -o run --output-format csv -- tools/micro/fetch_calib $mode \
            > $OUT/${mode}_$name.log 2>&1
        rc=$?
        echo "$mode $name rc=$rc"
        if [ $rc -ne 0 ]; then tail -5 $OUT/${mode}_$name.log; exit $rc; fi
    done
done
echo calib-ok
