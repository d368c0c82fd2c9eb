"""Interleaved A/B of run-time settings on one rank's share of C3 (GPU): kernel ms per variant.

    python tools/part_ab.py 8 1024 3 "sum:" "max:PT_TILE_KEY_MAX=1"

Each variant keeps its own film (its own tile costs and launch order), so a setting that changes
the longest-first order is measured with the order it produced itself.  Round 0 is the warmup
that measures the first tile costs.  Images of all variants must agree bit for bit.
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402


def main():
    n, spp, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    variants = []
    for v in sys.argv[4:]:
        name, _, envs = v.partition(":")
        variants.append((name, dict(e.split("=", 1) for e in envs.split(",") if e)))
    p = ptamd.Preset(os.environ.get("AB_PRESET", "bunny_cornell"))
    scene = ptamd.Scene(p.objects, p.materials)
    films = {name: ptamd.Film(p.width, p.height, 1, stripe_height=8, n_parts=n, part=0) for name, _ in variants}
    times = {name: [] for name, _ in variants}
    ref = None
    base_env = dict(os.environ)
    for r in range(rounds + 1):
        for name, env in variants:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(env)
            img, st = ptamd.render(scene, films[name], p.camera, spp, p.max_depth, rng=ptamd.RNG_SAMPLE)
            if ref is None:
                ref = img.copy()
            elif not (img.view("u4") == ref.view("u4")).all():
                raise SystemExit(f"variant {name}: image differs")
            if r > 0:
                times[name].append(st.kernel_ms)
    for name, _ in variants:
        t = times[name]
        print(json.dumps({"n_parts": n, "variant": name, "median_ms": round(statistics.median(t), 2),
                          "min_ms": round(min(t), 2), "all": [round(x, 2) for x in t]}), flush=True)


if __name__ == "__main__":
    main()
