# Instanced C5 with and without partial re-braiding (interleaved, twice).  GPU box.
set -e
for r in 1 2; do
for v in ${LEVELS:-1 0}; do
  PT_INST_REBRAID=$v timeout -k 10 150 python -u bench.py --config c5i --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abi_${v}_$r.json 2>gpurun_out/abi_${v}_$r.err
  python3 -c "import json;d=json.load(open('gpurun_out/abi_${v}_$r.json'));print('c5i rebraid $v $r', round(d['value'],1), round(d['ms_per_step'],2), flush=True)"
done; done
