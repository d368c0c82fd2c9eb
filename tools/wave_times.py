"""Per-wave timeline of one render launch (diagnostic; PT_WAVE_TIMES).
usage: python tools/wave_times.py [config] [spp] [out.bin]  -> prints a load-balance summary."""
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402


def analyse(t: np.ndarray, slots: int) -> dict:
    start, end = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    t0 = start.min()
    start, end = start - t0, end - t0
    span = end.max()
    dur = end - start
    # concurrency timeline at 1000 sample points
    grid = np.linspace(0, span, 1000)
    conc = np.array([((start <= x) & (end > x)).sum() for x in grid])
    return {"waves": len(t), "span_ms": span / 1e5, "mean_wave_ms": dur.mean() / 1e5, "max_wave_ms": dur.max() / 1e5,
            "util_vs_slots": float(dur.sum() / (span * slots)), "peak_concurrency": int(conc.max()),
            "time_at_<90%_peak": float((conc < 0.9 * conc.max()).mean()),
            "time_at_<50%_peak": float((conc < 0.5 * conc.max()).mean()),
            "last_start_ms": start.max() / 1e5,
            "end_pct_ms": {str(q): float(np.percentile(end, q) / 1e5) for q in (1, 10, 50, 90, 99, 100)},
            "xcc_span_ms": [float((end[(t[:, 2] >> 32) == x].max() - start[(t[:, 2] >> 32) == x].min()) / 1e5)
                            for x in range(8) if ((t[:, 2] >> 32) == x).any()]}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "gpurun_out", f"wave_times_{cfg}.bin")
    name = {"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}[cfg]
    p = ptamd.Preset(name)
    scene = ptamd.Scene(p.objects, p.materials)
    nparts = int(os.environ.get("NPARTS", "1"))   # one rank's share of an N-GPU frame
    film = ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=nparts, part=int(os.environ.get("PART", "0")))
    if int(os.environ.get("WARM", "0")):   # one launch first: the next one runs longest-first
        ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_SAMPLE if os.environ.get("RNG") == "sample"
                     else ptamd.RNG_COMPAT, chunk=int(os.environ.get("CHUNK", "0")))
        film.reset()
    os.environ["PT_WAVE_TIMES"] = out
    rng = ptamd.RNG_SAMPLE if os.environ.get("RNG") == "sample" else ptamd.RNG_COMPAT
    rgb, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=rng, chunk=int(os.environ.get("CHUNK", "0")))
    t = np.fromfile(out, dtype=np.uint64).reshape(-1, 3)
    print(json.dumps({"config": cfg, "spp": spp, "kernel_ms": st.kernel_ms, **analyse(t, 5 * 1024)}))


if __name__ == "__main__":
    main()
