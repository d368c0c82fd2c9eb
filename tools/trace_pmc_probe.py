"""Diagnostic (GPU, under rocprofv3 --pmc): one wide-tree closest-hit launch of C5 rays from one
origin in the camera's direction cone, then one of incoherent rays, 4 M each (tools/trace_probe.py)."""
import os
import sys

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

n = 4_000_000
p = pt.Preset("bunny_field")
scene = pt.Scene(p.objects, p.materials)
rng = np.random.default_rng(1)
cam = pt.camera_to_array(p.camera)
pos, ll, hor, ver = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
u, v = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
lo, hi = p.objects["v"][:, :3].min(0), p.objects["v"][:, :3].max(0)
cone = np.zeros(n, pt.RAY_DTYPE)
cone["o"] = np.array([pos[0], pos[1], lo[2] + 5.0], np.float32)
cone["d"] = ll + u[:, None] * hor + v[:, None] * ver - pos
inco = np.zeros(n, pt.RAY_DTYPE)
inco["o"] = rng.uniform(lo + 0.02 * (hi - lo), hi - 0.02 * (hi - lo), (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
inco["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
for name, r in (("cone", cone), ("incoherent", inco)):
    _, st = scene.trace(r, kernel=pt.KERNEL_WIDE)
    print(name, f"{st.kernel_ms:.3f} ms", st.node_visits / n, st.tri_tests / n, flush=True)
