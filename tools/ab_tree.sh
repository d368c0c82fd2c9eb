# Wide-tree A/B at the bench configs: host SAH tree with and without the small-subtree sweep, and
# the device SAH tree (interleaved, twice).  GPU box: bash tools/ab_tree.sh [configs...]
set -e
cfgs=${*:-c3 c5 c2}
for r in 1 2; do
for cfg in $cfgs; do
for v in host_sweep host_bins device; do
  case $v in
    host_sweep) env="PT_WIDE_BUILD=host PT_WIDE_SWEEP=64" ;;
    host_bins) env="PT_WIDE_BUILD=host PT_WIDE_SWEEP=0" ;;
    device) env="PT_WIDE_BUILD=device" ;;
  esac
  env $env timeout -k 10 150 python -u bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abt_${cfg}_${v}_$r.json 2>gpurun_out/abt_${cfg}_${v}_$r.err
  python3 -c "import json;d=json.load(open('gpurun_out/abt_${cfg}_${v}_$r.json'));print('$cfg $v $r', round(d['value'],1), round(d['ms_per_step'],2), flush=True)"
done; done; done
