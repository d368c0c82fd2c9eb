"""Compare the wide-tree kernel with the reference-order kernel on full frames (GPU only).

Both kernels render the same image except where the reference's own box test is inconsistent
with its primitive test (a grazing hit whose box entry rounds past the hit): this script counts
the pixels that differ and the rays per frame, per configuration.

    python tools/wide_vs_ref.py [c3|c2|c5] [spp] [rng]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

NAMES = {"c3": "bunny_cornell", "c2": "cornell", "c5": "bunny_field"}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rng = pt.RNG_SAMPLE if (len(sys.argv) <= 3 or sys.argv[3] == "sample") else pt.RNG_COMPAT
    p = pt.Preset(NAMES[cfg])
    s = pt.Scene(p.objects, p.materials, device=0)
    out = {}
    for name, k in (("wavefront", pt.KERNEL_WAVEFRONT), ("wide", pt.KERNEL_WIDE)):
        f = pt.Film(p.width, p.height, 1, device=0)
        rgb, st = pt.render(s, f, p.camera, spp, p.max_depth, kernel=k, rng=rng)
        out[name] = (rgb, st)
        print(f"{name:10s} rays {st.rays} visits {st.node_visits} tris {st.tri_tests} kernel {st.kernel_ms:.1f} ms",
              flush=True)
    a, b = out["wavefront"][0], out["wide"][0]
    diff = np.abs(a.astype(np.float64) - b.astype(np.float64)).max(axis=1)
    nd = int((diff > 0).sum())
    print(f"{cfg} spp {spp}: pixels differing {nd} of {len(diff)} (max |diff| {diff.max():.3g}); "
          f"rays {out['wavefront'][1].rays} vs {out['wide'][1].rays} "
          f"({out['wide'][1].rays - out['wavefront'][1].rays:+d})")


if __name__ == "__main__":
    main()
