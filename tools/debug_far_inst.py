"""Debug aid: far-camera instanced render vs flattened (trace of the camera rays, 1-bounce frames)."""
import sys
import os

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ptamd as pt  # noqa: E402
from helpers import rays_to_struct  # noqa: E402

w, h = 96, 64
ip = pt.InstancedPreset("bunny_field", w, h)
fp = pt.Preset("bunny_field", w, h)
lo, hi = fp.objects["v"][:, :3].min(0), fp.objects["v"][:, :3].max(0)
c = (lo + hi) / 2
ext = float((hi - lo).max())
dist = float(sys.argv[1]) if len(sys.argv) > 1 else 40.0
cam = pt.camera_make(c + np.array([0.3, 0.5, -1.0], np.float32) * dist * ext, c, 1.2, w / h)
si = pt.Scene.instanced(ip.objects, ip.mesh_first, ip.mesh_count, ip.instances, ip.materials)
sf = pt.Scene(fp.objects, fp.materials)
ca = pt.camera_to_array(cam)
org, ll, hor, ver = ca[0:3], ca[3:6], ca[6:9], ca[9:12]
ys, xs = np.mgrid[0:h, 0:w]
u = ((xs + 0.5) / w).reshape(-1, 1)
v = ((ys + 0.5) / h).reshape(-1, 1)
rays = np.zeros((w * h, 6), np.float32)
rays[:, :3] = org
rays[:, 3:] = ll + u * hor + v * ver - org
r = rays_to_struct(rays, pt.RAY_DTYPE)
gi, _ = si.trace(r, kernel=pt.KERNEL_WIDE)
gf, _ = sf.trace(r, kernel=pt.KERNEL_WIDE)
print("trace: hit frac inst %.4f flat %.4f, agree %.4f, same obj %.4f" % (
    gi["hit"].mean(), gf["hit"].mean(), (gi["hit"] == gf["hit"]).mean(),
    ((gi["obj"] == gf["obj"]) | (gi["hit"] == 0)).mean()))
for depth in (1, 2, 16):
    ri, sti = pt.render(si, pt.Film(w, h, 3), cam, 4, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    rf, stf = pt.render(sf, pt.Film(w, h, 3), cam, 4, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    print(f"depth {depth}: mean inst {ri.mean(0)} flat {rf.mean(0)}, rays {sti.rays} {stf.rays}, "
          f"pixels differing {(np.abs(ri - rf).max(1) > 0.05).mean():.4f}")
print("scene box", lo, hi, "ext", ext, "cam", org)
