"""Diagnostic (GPU): closest-hit rate of C5-style camera rays under variations -- raw camera
directions (unnormalised, as camera::get_ray makes them), the same directions normalised, and the
same directions from an origin inside the scene box -- on the wide tree (queued kernel).

    python tools/trace_probe.py [preset] [n_rays_millions]
"""
import os
import sys

import numpy as np
import torch  # noqa: F401  (device init order as in the other tools)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bunny_field"
n = int(float(sys.argv[2]) * 1e6) if len(sys.argv) > 2 else 4_000_000
p = pt.Preset(name)
scene = pt.Scene(p.objects, p.materials)
rng = np.random.default_rng(1)
cam = pt.camera_to_array(p.camera)
pos, ll, hor, ver = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
u, v = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
d = (ll + u[:, None] * hor + v[:, None] * ver - pos).astype(np.float32)
lo, hi = p.objects["v"][:, :3].min(0), p.objects["v"][:, :3].max(0)
variants = {
    "raw": (pos, d),
    "normalised": (pos, d / np.linalg.norm(d, axis=1, keepdims=True)),
    "origin z=lo+5": (np.array([pos[0], pos[1], lo[2] + 5.0], np.float32), d),
    "sorted by pixel": None,
}
for vname, val in variants.items():
    r = np.zeros(n, pt.RAY_DTYPE)
    if val is None:   # the raw rays in scanline order of their image position (coherent lanes)
        order = np.lexsort((u, np.floor(v * 1080)))
        r["o"] = pos
        r["d"] = d[order]
    else:
        r["o"], r["d"] = val
    for k in (pt.KERNEL_WIDE, pt.KERNEL_WAVEFRONT):
        best = None
        for _ in range(3):
            hits, st = scene.trace(r, kernel=k)
            best = st if best is None or st.kernel_ms < best.kernel_ms else best
        print(f"{name} {vname:16s} {'wide' if k == pt.KERNEL_WIDE else 'binary':6s} {n / best.kernel_ms / 1e3:7.0f} Mray/s  "
              f"visits/ray {best.node_visits / n:5.2f}  tests/ray {best.tri_tests / n:5.2f}  hit {hits['hit'].mean():.3f}",
              flush=True)
