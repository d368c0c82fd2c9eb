# bench.py A/B of library builds (PT_LIB) at the bench configs, interleaved, twice.
#   LIBS="base:path-tracer-cuda-opengl_amd/libpt.so x:path-tracer-cuda-opengl_amd/variants/libpt_x.so" CFGS="c3 c5" bash tools/ab_libs_bench.sh
set -e
for r in 1 2; do
for cfg in ${CFGS:-c3 c5}; do
for spec in $LIBS; do
  name=${spec%%:*}; lib=${spec#*:}
  PT_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-compat --no-interactive > gpurun_out/abl_${cfg}_${name}_$r.json 2>gpurun_out/abl_${cfg}_${name}_$r.err
  python3 -c "import json;d=json.load(open('gpurun_out/abl_${cfg}_${name}_$r.json'));print('$cfg $name $r', round(d['value'],1), round(d['ms_per_step'],2), d['scene_build'].get('wide_tree_host_ms'), flush=True)"
done; done; done
