"""Interactive-mode frames only (bench.py's `interactive` loop: camera move, clear, accumulate spp
samples, RGBA8 surface), for rocprofv3 --kernel-trace: where a low-spp frame's time goes.
usage: python tools/interactive_prof.py [config] [spp] [frames]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

NAMES = {"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    p = ptamd.Preset(NAMES[cfg])
    scene = ptamd.Scene(p.objects, p.materials)
    film = ptamd.Film(p.width, p.height, 1)
    buf = torch.empty((p.width * p.height * 4,), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    cam = ptamd.Camera.from_buffer_copy(bytes(p.camera))
    for it in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            ptamd.camera_move(cam, (0, 2, 1, 3)[k % 4], 0.01)
            film.clear(stream.cuda_stream)
            ptamd.render(scene, film, cam, spp, p.max_depth, out=buf.data_ptr(), stream=stream.cuda_stream,
                         rng=ptamd.RNG_SAMPLE, accumulate=True, out_format=ptamd.OUT_RGBA8_SURFACE, wait=False)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    st = film.stats()
    print(json.dumps({"config": cfg, "spp": spp, "fps": n / el, "ms_per_frame": el / n * 1e3,
                      "rays_per_frame": st.rays, "kernel_ms": st.kernel_ms}))


if __name__ == "__main__":
    main()
