set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -k sample_mode_options > gpurun_out/t.log 2>&1; echo rc=$?; tail -2 gpurun_out/t.log
for m in "compat 0" "sample 64" "sample 256" "sample 1024"; do set -- $m
RNG=$1 CHUNK=$2 timeout -k 10 200 python tools/wave_times.py c3 1024 gpurun_out/wt.bin || exit 1
done
