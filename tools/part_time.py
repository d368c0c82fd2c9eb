"""Frame time of one rank's share (part p of n stripes) on one GPU: predicts the multi-GPU frame
time without a multi-GPU box.  usage: python tools/part_time.py [n_parts] [compat|sample] [spp]
ALL=1 times every part (max / mean share time: the balance across ranks); CFG=c2|c3|c5."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
mode = sys.argv[2] if len(sys.argv) > 2 else "sample"
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
rng = ptamd.RNG_SAMPLE if mode == "sample" else ptamd.RNG_COMPAT
p = ptamd.Preset({"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}[os.environ.get("CFG", "c3")])
scene = ptamd.Scene(p.objects, p.materials)
parts = range(n) if os.environ.get("ALL") else sorted({0, n // 2, n - 1})
best = []
for part in parts:
    f = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=n, part=part)
    out = torch.empty((f.n_pixels * 3,), dtype=torch.float32, device="cuda")
    times, kms = [], []
    for it in range(3):
        f.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, st = ptamd.render(scene, f, p.camera, spp, p.max_depth, out=out.data_ptr(), rng=rng,
                             flags=ptamd.IDENTITY_ORDER if os.environ.get("IDENTITY") else 0,
                             chunk=int(os.environ.get("CHUNK", "0")))
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        kms.append(st.kernel_ms)
    best.append(min(kms[1:]))   # (the first launch measures tile costs for the longest-first order)
    print(json.dumps({"n_parts": n, "part": part, "mode": mode, "ms": [round(t * 1e3, 1) for t in times],
                      "kernel_ms": [round(k, 1) for k in kms], "rays": st.rays}), flush=True)
print(json.dumps({"n_parts": n, "parts_timed": len(best), "max_kernel_ms": max(best),
                  "mean_kernel_ms": sum(best) / len(best), "max_over_mean": max(best) / (sum(best) / len(best))}),
      flush=True)
