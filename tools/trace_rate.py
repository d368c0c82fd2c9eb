"""Closest-hit throughput of pt_trace_closest_device (the hitBvh replacement on device-resident
rays; GPU only): C3 scene, camera rays and incoherent rays (random origins inside the Cornell box,
random directions), wide tree vs the binary LBVH in the reference's order.

    python tools/trace_rate.py [n_rays_millions]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

n = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 16_000_000
name = sys.argv[2] if len(sys.argv) > 2 else "bunny_cornell"
p = pt.Preset(name)
scene = pt.Scene(p.objects, p.materials)
rng = np.random.default_rng(1)
cam = pt.camera_to_array(p.camera)   # origin (pos), lower-left, horizontal, vertical
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
dev = torch.device("cuda", 0)
hits = torch.empty(n * pt.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
for name, rays in (("camera", camera), ("incoherent", inco)):
    rd = torch.from_numpy(rays.view(np.uint8)).to(dev)
    for kname, k, stride in (("wide", pt.KERNEL_WIDE, "0"), ("wide/stride", pt.KERNEL_WIDE, "1"),
                             ("binary", pt.KERNEL_WAVEFRONT, "0"), ("binary/stride", pt.KERNEL_WAVEFRONT, "1")):
        os.environ["PT_TRACE_STRIDE"] = stride
        best = None
        for _ in range(3):
            st = scene.trace_device(rd.data_ptr(), n, hits.data_ptr(), kernel=k)
            best = st if best is None or st.kernel_ms < best.kernel_ms else best
        hit = hits.cpu().numpy().view(pt.HIT_DTYPE)["hit"].mean()
        print(f"{name:10s} {kname:13s} {n / best.kernel_ms / 1e3:9.0f} Mray/s  {best.kernel_ms:8.2f} ms  "
              f"visits/ray {best.node_visits / n:5.2f}  prims/ray {(best.tri_tests + best.sphere_tests) / n:5.2f}  "
              f"hit {hit:.3f}", flush=True)
