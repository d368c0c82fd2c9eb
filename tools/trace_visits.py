"""Diagnostic (GPU, a -DPT_TRACE_DIAG_VISITS=1 build loaded with PT_LIB: each hit record's `mat`
holds the query's wide node visits): the per-query visit distribution of C5 rays from one origin in
the camera's direction cone, camera rays and incoherent rays, with the longest queries listed.

    PT_LIB=.../variants/libpt_visits.so python tools/trace_visits.py [n_rays_millions]
"""
import os
import sys

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

n = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 4_000_000
p = pt.Preset("bunny_field")
scene = pt.Scene(p.objects, p.materials)
rng = np.random.default_rng(1)
cam = pt.camera_to_array(p.camera)
pos, ll, hor, ver = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
u, v = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
lo, hi = p.objects["v"][:, :3].min(0), p.objects["v"][:, :3].max(0)
d = (ll + u[:, None] * hor + v[:, None] * ver - pos).astype(np.float32)
cone = np.zeros(n, pt.RAY_DTYPE)
cone["o"] = np.array([pos[0], pos[1], lo[2] + 5.0], np.float32)
cone["d"] = d
camera = np.zeros(n, pt.RAY_DTYPE)
camera["o"] = pos
camera["d"] = d
inco = np.zeros(n, pt.RAY_DTYPE)
inco["o"] = rng.uniform(lo + 0.02 * (hi - lo), hi - 0.02 * (hi - lo), (n, 3)).astype(np.float32)
g = rng.normal(size=(n, 3)).astype(np.float32)
inco["d"] = g / np.linalg.norm(g, axis=1, keepdims=True)
for name, r in (("cone", cone), ("camera", camera), ("incoherent", inco)):
    hits, st = scene.trace(r, kernel=pt.KERNEL_WIDE)
    vis = hits["mat"].astype(np.int64)
    assert vis.sum() == st.node_visits, (vis.sum(), st.node_visits)
    q = np.percentile(vis, [50, 99, 99.9, 99.99])
    print(f"{name:10s} {st.kernel_ms:7.3f} ms  visits mean {vis.mean():.2f}  p50/p99/p99.9/p99.99 {q}  max {vis.max()}  "
          f">100: {(vis > 100).sum()}  >1000: {(vis > 1000).sum()}", flush=True)
    for i in np.argsort(vis)[-5:][::-1]:
        print(f"    ray {i}: visits {vis[i]}  o {r['o'][i]}  d {r['d'][i]}  hit {hits['hit'][i]} t {hits['t'][i]}", flush=True)
