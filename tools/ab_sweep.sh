set -e
for r in 1 2; do
for cfg in c3 c5; do
for sw in 0 8 16 32; do
  PT_WIDE_BUILD=host PT_WIDE_SWEEP=$sw timeout -k 10 150 python -u bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abs_${cfg}_${sw}_$r.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/abs_${cfg}_${sw}_$r.json'));print('$cfg sweep $sw $r', round(d['value'],1), round(d['ms_per_step'],2), flush=True)"
done; done; done
