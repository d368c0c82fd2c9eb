"""Render one frame (profiling target).  usage: python tools/one_frame.py [c2|c3|c5|c5i] [spp] [compat|sample] [chunk]
REPEAT=n renders n frames (later launches use the measured tile costs) and reports the fastest.
NPARTS=n PART=k render one rank's share of an n-GPU frame (8-row stripes, stripe s on part s % n)."""
import hashlib
import json
import os
import sys

import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

cfg = os.environ.get("CFG") or (sys.argv[1] if len(sys.argv) > 1 else "c3")
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rng = ptamd.RNG_SAMPLE if len(sys.argv) > 3 and sys.argv[3] == "sample" else ptamd.RNG_COMPAT
chunk = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if cfg == "c5i":   # the instanced bunny field (two-level tree)
    p = ptamd.InstancedPreset("bunny_field")
    scene = ptamd.Scene.instanced(p.objects, p.mesh_first, p.mesh_count, p.instances, p.materials)
else:
    p = ptamd.Preset({"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field", "c5x4": "bunny_field_x4"}[cfg])
    scene = ptamd.Scene(p.objects, p.materials)
film = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=int(os.environ.get("NPARTS", "1")),
                  part=int(os.environ.get("PART", "0")))
best = None
digest = None
for _ in range(int(os.environ.get("REPEAT", "1"))):   # later launches use measured tile costs
    film.reset()
    img, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=rng, chunk=chunk)
    digest = hashlib.sha1(img.tobytes()).hexdigest()[:16]   # same for every library build that renders the same frame
    if best is None or st.kernel_ms < best.kernel_ms:
        best = st
st = best
print(json.dumps({"cfg": cfg, "spp": spp, "kernel_ms": st.kernel_ms, "rays": st.rays, "node_visits": st.node_visits,
                  "tri_tests": st.tri_tests, "image": digest}))
