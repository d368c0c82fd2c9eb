#!/bin/bash
# Bench + rocprofv3 session on the GPU box (run via gpurun).  TAG names the output dir.
#  1. python bench.py (the driver's default command)          -> gpurun_out/$TAG/bench.json
#  2. rocprofv3 --kernel-trace --stats of the same frames (without the CPU baseline and the
#     interactive-mode frames, whose 1-16 spp launches would mix into the render kernel's average,
#     and without the `pipelined` frames, whose overlapping launches last longer than a frame)
#                                                               -> gpurun_out/$TAG/trace/
#  3. separate --pmc passes (FETCH_SIZE | WRITE_SIZE | TCC hit/miss | SQ | VALU instructions) on one frame
#     after one warmup frame of the same kernel (so the counted launch is a steady-state one: sample
#     mode's first launch on a film also counts every task's rays for the tile order, a 4th atomic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:-}
PMC_ARGS=${PMC_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-compat --no-interactive --no-pipelined}
TRACE_ARGS=${TRACE_ARGS:---no-cpu-baseline --no-interactive --no-pipelined}
step() {  # name, limit, command...
    local name=$1 lim=$2; shift 2
    timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-400
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench 600 python bench.py $BENCH_ARGS
grep '^{' $OUT/bench.log > $OUT/bench.json
step trace 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $TRACE_ARGS $BENCH_ARGS
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS $BENCH_ARGS
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PMC_ARGS $BENCH_ARGS
step pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o run --output-format csv -- python3 bench.py $PMC_ARGS $BENCH_ARGS
step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $PMC_ARGS $BENCH_ARGS
step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $OUT/pmc_valu -o run --output-format csv -- python3 bench.py $PMC_ARGS $BENCH_ARGS
echo all-ok
