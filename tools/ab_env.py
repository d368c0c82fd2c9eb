"""Interleaved A/B of run-time settings in one process (GPU): median kernel ms per variant.

    python tools/ab_env.py c3 256 3 "base:" "l32:PT_LEAF_BATCH=32" "l32s24:PT_LEAF_BATCH=32,PT_SHADE_BATCH=24"

Each round renders every variant once (sample mode, the default kernel unless PT_RENDER_KERNEL is
in the variant), so clock drift hits all variants alike.  Images must agree bit for bit.
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

NAMES = {"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field"}


def main():
    cfg, spp, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    variants = []
    for v in sys.argv[4:]:
        name, _, envs = v.partition(":")
        variants.append((name, dict(e.split("=", 1) for e in envs.split(",") if e)))
    rng = ptamd.RNG_COMPAT if os.environ.get("AB_RNG") == "compat" else ptamd.RNG_SAMPLE
    p = ptamd.Preset(NAMES[cfg])
    scene = ptamd.Scene(p.objects, p.materials)
    film = ptamd.Film(p.width, p.height, 1)
    times = {n: [] for n, _ in variants}
    ref = None
    base_env = dict(os.environ)
    for r in range(rounds + 1):   # round 0: warmup (tile costs, wide tree build)
        for name, env in variants:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(env)
            film.reset()
            img, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=rng)
            if ref is None:
                ref = img.copy()
            elif not (img.view("u4") == ref.view("u4")).all():
                raise SystemExit(f"variant {name}: image differs")
            if r > 0:
                times[name].append(st.kernel_ms)
    for name, _ in variants:
        t = times[name]
        print(json.dumps({"variant": name, "median_ms": statistics.median(t), "min_ms": min(t), "all": t}))


if __name__ == "__main__":
    main()
