# Sample-mode summation block (--chunk) A/B at the bench configs (interleaved, twice).
set -e
for r in 1 2; do
for cfg in ${CFGS:-c3 c5 c2}; do
for ch in ${CHUNKS:-16 32 64}; do
  timeout -k 10 150 python -u bench.py --config $cfg --chunk $ch --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abc_${cfg}_${ch}_$r.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/abc_${cfg}_${ch}_$r.json'));print('$cfg chunk $ch $r', round(d['value'],1), round(d['ms_per_step'],2), flush=True)"
done; done; done
