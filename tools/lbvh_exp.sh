set -e
for cfg in "c3 256" "c5 64" "c2 1024"; do
  for f in 1 2; do
    r=$(PT_WIDE_MAX_LEAF=$f PT_WIDE_FROM_LBVH=1 REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg sample | tail -1)
    echo "lbvh maxleaf=$f $cfg: $r"
  done
  r=$(PT_RENDER_KERNEL=wavefront REPEAT=3 timeout -k 5 200 python tools/one_frame.py $cfg sample | tail -1)
  echo "binary $cfg: $r"
done
