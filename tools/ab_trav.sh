# Host SAH node-visit weight (PT_WIDE_TRAV_COST) A/B at the bench configs (interleaved, twice).
set -e
for r in 1 2; do
for cfg in ${CFGS:-c3 c5}; do
for tc in ${TRAVS:-0.5 1 2}; do
  PT_WIDE_TRAV_COST=$tc timeout -k 10 150 python -u bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abtc_${cfg}_${tc}_$r.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/abtc_${cfg}_${tc}_$r.json'));print('$cfg trav $tc $r', round(d['value'],1), round(d['ms_per_step'],2), flush=True)"
done; done; done
