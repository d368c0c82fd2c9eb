"""Build one preset's LBVH (+ the device wide tree) a few times (profiling target).
usage: python tools/build_only.py [c2|c3|c5] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
p = pt.Preset({"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}[cfg])
flags = pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_WIDE_DEVICE
s = pt.Scene(p.objects, p.materials, flags=flags)
t = []
for _ in range(reps):
    s.build_bvh(flags)
    t.append(s.build_ms)
print(cfg, "build ms", [round(x, 2) for x in t], s.wide_info())
