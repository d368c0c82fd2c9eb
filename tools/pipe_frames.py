"""Frames in flight: K frames of a config rendered back to back on one stream (one film) vs
alternating between two films on two streams (a frame's first waves start while the previous
frame's last paths finish).  Wall time per frame; optionally one rank's share (N_PARTS, PART).

    python tools/pipe_frames.py [c3|c5|c2] [frames]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
name, spp = {"c2": ("cornell", 256), "c3": ("bunny_cornell", 1024), "c5": ("bunny_field", 512)}[cfg]
n_parts, part = int(os.environ.get("N_PARTS", "1")), int(os.environ.get("PART", "0"))
p = ptamd.Preset(name)
scene = ptamd.Scene(p.objects, p.materials)
films = [ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=n_parts, part=part) for _ in range(2)]
bufs = [torch.empty((films[0].n_pixels * 4,), dtype=torch.uint8, device="cuda") for _ in range(2)]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
for j in range(2):   # warm: tile costs, launch order
    for _ in range(2):
        ptamd.render(scene, films[j], p.camera, spp, p.max_depth, out=bufs[j].data_ptr(), stream=streams[j].cuda_stream,
                     rng=ptamd.RNG_SAMPLE, out_format=ptamd.OUT_RGBA8)
torch.cuda.synchronize()
res = {}
for rep in range(2):
    for pipes in (1, 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            j = k % pipes
            ptamd.render(scene, films[j], p.camera, spp, p.max_depth, out=bufs[j].data_ptr(),
                         stream=streams[j].cuda_stream, rng=ptamd.RNG_SAMPLE, out_format=ptamd.OUT_RGBA8, wait=False)
        torch.cuda.synchronize()
        res.setdefault(pipes, []).append((time.perf_counter() - t0) / K * 1e3)
same = torch.equal(bufs[0], bufs[1])
print(f"{cfg} parts {n_parts}: ms/frame one stream {min(res[1]):.2f}, two streams {min(res[2]):.2f} "
      f"({(1 - min(res[2]) / min(res[1])) * 100:.1f} % less); frames equal {same}", flush=True)
