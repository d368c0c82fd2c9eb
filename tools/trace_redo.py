"""Diagnostic (GPU, a -DPT_TRACE_DIAG_REDO=1 build loaded with PT_LIB): the share of closest-hit
queries that end in the reference-order redo (traceRefStackless) on the wide tree, for camera and
incoherent rays -- such a build counts them as sphere tests, so only scenes without spheres.

    PT_LIB=.../variants/libpt_redo.so python tools/trace_redo.py [preset] [n_rays_millions]
"""
import os
import sys

import numpy as np
import torch

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
camera = np.zeros(n, pt.RAY_DTYPE)
camera["o"] = pos
camera["d"] = ll + u[:, None] * hor + v[:, None] * ver - pos
inco = np.zeros(n, pt.RAY_DTYPE)
lo, hi = p.objects["v"][:, :3].min(0), p.objects["v"][:, :3].max(0)
inco["o"] = rng.uniform(lo + 0.02 * (hi - lo), hi - 0.02 * (hi - lo), (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
inco["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
for rname, rays in (("camera", camera), ("incoherent", inco)):
    hits, st = scene.trace(rays, kernel=pt.KERNEL_WIDE)
    print(f"{name} {rname:10s} redo share {st.sphere_tests / n:.4f}  wide visits/ray {st.node_visits / n:.2f}  "
          f"tri tests/ray {st.tri_tests / n:.2f}  {n / st.kernel_ms / 1e3:.0f} Mray/s  hit {hits['hit'].mean():.3f}",
          flush=True)
