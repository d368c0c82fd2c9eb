"""Holds a GPU context the way the pytest suite process does (torch + libpt, four torch streams with
work on each, a film and a small frame), then sleeps until killed.  Used by tools/queue_probe.sh."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

ss = [torch.cuda.Stream() for _ in range(int(os.environ.get("HOLD_STREAMS", "4")))]
xs = []
for s in ss:
    with torch.cuda.stream(s):
        xs.append(torch.ones(1 << 20, device="cuda") * 2)
p = ptamd.Preset("cornell", 64, 64)
scene = ptamd.Scene(p.objects, p.materials)
film = ptamd.Film(64, 64, 1)
ptamd.render(scene, film, p.camera, 4, 8, stream=ss[-1].cuda_stream)
torch.cuda.synchronize()
print("holder ready", flush=True)
time.sleep(float(os.environ.get("HOLD_S", "900")))
