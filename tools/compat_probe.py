"""Compat-mode critical path probe (diagnostic; PT_WAVE_TIMES, PT_COMPAT_GRID_LIMIT).

    python tools/compat_probe.py [c3] [spp] [limits...]

Frame 1 measures the tile costs (the launch order of the next frames).  Frame 2 is the full
frame with per-wave timestamps: its end-time percentiles and its longest waves (tile, start,
duration).  Then, for each limit k, a frame of only the first k waves of the launch order (the
longest tiles; the rest of the machine idle): the same waves' durations when they run alone, i.e.
how much of the loaded duration is the chains' own latency and how much is sharing the machine.
Env knobs of the library (PT_SPLIT_TILES, PT_SPLIT_WAYS, PT_PRIO_TILES, ...) apply to every frame.
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402


def frame(scene, film, p, spp, times=None, limit=0):
    for k in ("PT_WAVE_TIMES", "PT_COMPAT_GRID_LIMIT"):
        os.environ.pop(k, None)
    if times:
        os.environ["PT_WAVE_TIMES"] = times
    if limit:
        os.environ["PT_COMPAT_GRID_LIMIT"] = str(limit)
    film.reset()
    _, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_COMPAT)
    if not times:
        return st, None
    t = np.fromfile(times, dtype=np.uint64).reshape(-1, 3)
    return st, t


def summary(t, top=12):
    start, end = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    ok = end > 0
    t0 = start[ok].min()
    s, e = (start - t0) / 1e5, (end - t0) / 1e5   # 100 MHz realtime counter -> ms
    dur = e - s
    order = np.argsort(-dur * ok)
    longest = [{"wave": int(i), "tile": int(t[i, 2] & 0xffffffff), "start_ms": round(float(s[i]), 2),
                "dur_ms": round(float(dur[i]), 2)} for i in order[:top] if ok[i]]
    last = np.argsort(-e * ok)
    latest = [{"wave": int(i), "tile": int(t[i, 2] & 0xffffffff), "start_ms": round(float(s[i]), 2),
               "dur_ms": round(float(dur[i]), 2)} for i in last[:top] if ok[i]]
    # how long the machine runs below full occupancy: waves still running at the p-th end-time
    return {"waves": int(ok.sum()), "span_ms": float(e[ok].max()), "latest": latest,
            "start_pct_ms": {str(q): round(float(np.percentile(s[ok], q)), 1) for q in (50, 90, 99, 100)},
            "end_pct_ms": {str(q): round(float(np.percentile(e[ok], q)), 1) for q in (50, 90, 99, 99.9, 100)},
            "longest": longest}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    limits = [int(x) for x in sys.argv[3:]] or [256]
    p = ptamd.Preset({"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}[cfg])
    scene = ptamd.Scene(p.objects, p.materials)
    film = ptamd.Film(p.width, p.height, 1, stripe_height=8)
    tmp = tempfile.mkdtemp()
    st0, _ = frame(scene, film, p, spp)   # costs -> the launch order
    st, t = frame(scene, film, p, spp, os.path.join(tmp, "full.bin"))
    full = summary(t)
    print(json.dumps({"cfg": cfg, "spp": spp, "first_ms": st0.kernel_ms, "kernel_ms": st.kernel_ms, "full": full}),
          flush=True)
    for lim in limits:
        # (the order of the next launch is made from this partial frame's costs: re-measure first)
        frame(scene, film, p, spp)
        stl, tl = frame(scene, film, p, spp, os.path.join(tmp, f"lim{lim}.bin"), limit=lim)
        sub = summary(tl)
        # the same tiles in the full frame (longest of the tile's waves)
        tiles = t[:, 2] & 0xffffffff
        dur = (t[:, 1].astype(np.int64) - t[:, 0].astype(np.int64)) / 1e5
        loaded = [round(float(dur[tiles == w["tile"]].max()), 2) if (tiles == w["tile"]).any() else None
                  for w in sub["longest"]]
        print(json.dumps({"limit": lim, "kernel_ms": stl.kernel_ms, "alone": sub,
                          "same_tiles_loaded_dur_ms": loaded}), flush=True)


if __name__ == "__main__":
    main()
