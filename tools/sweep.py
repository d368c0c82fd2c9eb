"""Scheduler sweep on the GPU box: one process, one scene, many (kernel, thresholds) settings.
usage: python tools/sweep.py [config] [spp] ; prints one JSON line per setting."""
import json
import os
import sys
import time

import torch  # noqa: F401  (same HIP runtime as bench.py)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

name = {"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}[sys.argv[1] if len(sys.argv) > 1 else "c3"]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 128
settings = [("simple", 16, 24), ("wavefront", 8, 16)] + [("wide", l, s) for l, s in
            [(4, 12), (6, 16), (8, 16), (8, 24), (12, 16), (12, 24), (16, 24), (16, 32)]]
if len(sys.argv) > 3:
    settings = [tuple(x.split(":")[:1]) + tuple(int(v) for v in x.split(":")[1:]) for x in sys.argv[3].split(",")]
p = ptamd.Preset(name)
scene = ptamd.Scene(p.objects, p.materials)
film = ptamd.Film(p.width, p.height, 1)
rgb = None
for k, lb, sb in settings:
    os.environ.update(PT_RENDER_KERNEL=k, PT_LEAF_BATCH=str(lb), PT_SHADE_BATCH=str(sb))
    rgb, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, out=rgb)   # warm
    t = time.perf_counter()
    rgb, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, out=rgb)
    el = time.perf_counter() - t
    print(json.dumps({"kernel": k, "leaf": lb, "shade": sb, "spp": spp, "scene": name,
                      "Mray_s": st.rays / (st.kernel_ms * 1e3), "kernel_ms": st.kernel_ms, "wall_s": el,
                      "GBs_algo": st.algo_bytes / st.kernel_ms / 1e6}), flush=True)
