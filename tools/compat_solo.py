"""The compat frame's longest tile alone on the GPU, split into `ways` waves of 64 / ways pixels
(diagnostic: PT_SPLIT_TILES=1, PT_SPLIT_WAYS, PT_COMPAT_GRID_LIMIT, PT_WAVE_TIMES; with a PT_DIAG
library and PT_ITER_STATS=1 the launch's step counts and cycles go to stderr).

    python tools/compat_solo.py [spp] [ways...]

Per ways: one full frame (its wave durations give the next launch's longest-first order), then a
launch of only the first tile of that order, split; prints each of its waves' duration."""
import json
import os
import sys
import tempfile

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    ways = [int(x) for x in sys.argv[2:]] or [2, 4, 8]
    p = ptamd.Preset("bunny_cornell")
    scene = ptamd.Scene(p.objects, p.materials)
    film = ptamd.Film(p.width, p.height, 1, stripe_height=8)
    tmp = tempfile.mkdtemp()
    stats = os.environ.pop("PT_ITER_STATS", None)
    for w in ways:
        os.environ.update(PT_SPLIT_WAYS=str(w), PT_SPLIT_TILES="1")
        for k in ("PT_WAVE_TIMES", "PT_COMPAT_GRID_LIMIT", "PT_ITER_STATS"):
            os.environ.pop(k, None)
        film.reset()
        _, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_COMPAT)
        path = os.path.join(tmp, f"w{w}.bin")
        os.environ.update(PT_WAVE_TIMES=path, PT_COMPAT_GRID_LIMIT=str(w))
        if stats:
            os.environ["PT_ITER_STATS"] = stats
        film.reset()
        sys.stderr.write(f"[solo] ways {w}\n")
        sys.stderr.flush()
        _, sl = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_COMPAT)
        t = np.fromfile(path, dtype=np.uint64).reshape(-1, 3)
        dur = [round(float((int(a[1]) - int(a[0])) / 1e5), 2) for a in t if a[1] > 0]
        print(json.dumps({"ways": w, "full_frame_ms": st.kernel_ms, "solo_kernel_ms": sl.kernel_ms,
                          "tile": int(t[0, 2] & 0xffffffff), "wave_ms": dur, "solo_rays": sl.rays}), flush=True)


if __name__ == "__main__":
    main()
