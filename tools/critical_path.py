"""Critical-path probe: render single 8-row stripes of C3 (GPU nearly idle) to measure how long
the slowest pixels' sequential sample chains take without contention."""
import json
import os
import sys

import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

p = ptamd.Preset("bunny_cornell")
scene = ptamd.Scene(p.objects, p.materials)
for kern, kname in ((ptamd.KERNEL_WAVEFRONT, "wavefront"), (ptamd.KERNEL_WIDE, "wide"), (ptamd.KERNEL_SIMPLE, "simple")):
    for stripe in (9, 12):   # rows 72-79 and 96-103 hold the slowest pixels
        film = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=135, part=stripe)
        _, st = ptamd.render(scene, film, p.camera, p.spp, p.max_depth, kernel=kern)
        print(json.dumps({"kernel": kname, "stripe": stripe, "rows": [int(film.rows[0]), int(film.rows[-1])],
                          "kernel_ms": st.kernel_ms, "rays": st.rays}), flush=True)
for parts in (2, 4, 8):   # one rank's share of an N-GPU frame, alone on this GPU
    film = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=parts, part=1)
    _, st = ptamd.render(scene, film, p.camera, p.spp, p.max_depth)
    film2 = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=parts, part=1)
    _, st2 = ptamd.render(scene, film2, p.camera, p.spp, p.max_depth)   # costs known -> LPT order
    _, st3 = ptamd.render(scene, film2, p.camera, p.spp, p.max_depth)
    print(json.dumps({"parts": parts, "part": 1, "kernel_ms": [st.kernel_ms, st2.kernel_ms, st3.kernel_ms],
                      "rays": st.rays}), flush=True)
