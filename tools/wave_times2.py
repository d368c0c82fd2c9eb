"""LPT diagnostic: C3 @1024spp rendered 3 times from the same initial streams (identity order,
then longest-first with 0 and with the default priority tiles); per-wave timeline of each."""
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"), os.path.join(REPO, "tools")]
import ptamd  # noqa: E402
from wave_times import analyse  # noqa: E402

p = ptamd.Preset("bunny_cornell")
scene = ptamd.Scene(p.objects, p.materials)
film = ptamd.Film(p.width, p.height, 1)
for label, prio in (("identity", "0"), ("lpt_noprio", "0"), ("lpt_prio1024", "1024")):
    out = os.path.join(REPO, "gpurun_out", f"wt_{label}.bin")
    os.environ.update(PT_WAVE_TIMES=out, PT_PRIO_TILES=prio)
    film.reset()
    rgb, st = ptamd.render(scene, film, p.camera, p.spp, p.max_depth)
    t = np.fromfile(out, dtype=np.uint64).reshape(-1, 3)
    print(json.dumps({"label": label, "kernel_ms": st.kernel_ms, "Mray_s": st.rays / st.kernel_ms / 1e3,
                      **analyse(t, 5 * 1024)}), flush=True)
