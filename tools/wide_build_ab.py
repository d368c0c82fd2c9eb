"""Device-built wide trees (PT_BVH_WIDE_DEVICE: binned SAH, PLOC) vs host-built (binned SAH):
build time, tree shape, frame time and frame equality.  GPU only.

    [AB_MODES=host,sah,ploc] python tools/wide_build_ab.py [c2|c3|c5 ...] [spp]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd as pt  # noqa: E402

NAMES = {"c3": "bunny_cornell", "c2": "cornell", "c5": "bunny_field"}
SPP = {"c2": 256, "c3": 64, "c5": 16}
cfgs = [a for a in sys.argv[1:] if a in NAMES] or ["c2", "c3", "c5"]
spp_arg = [int(a) for a in sys.argv[1:] if a.isdigit()]

for cfg in cfgs:
    p = pt.Preset(NAMES[cfg])
    spp = spp_arg[0] if spp_arg else SPP[cfg]
    out = {}
    for mode in os.environ.get("AB_MODES", "host,sah,ploc").split(","):
        os.environ["PT_WIDE_DEVICE_BUILDER"] = mode
        flags = pt.PT_BVH_ORIGIN_BOUNDS | (pt.PT_BVH_WIDE_DEVICE if mode != "host" else 0)
        s = pt.Scene(p.objects, p.materials, flags=flags)
        builds = []
        for _ in range(3):
            t0 = time.perf_counter()
            s.build_bvh(flags)
            builds.append((time.perf_counter() - t0) * 1e3)
        best = None
        img = None
        for _ in range(3):
            f = pt.Film(p.width, p.height, 1)
            im, st = pt.render(s, f, p.camera, spp, p.max_depth, rng=pt.RNG_SAMPLE, kernel=pt.KERNEL_WIDE)
            if best is None or st.kernel_ms < best.kernel_ms:
                best, img = st, im
        wi = s.wide_info()
        out[mode] = img
        print(f"{cfg} {mode:6s} lbvh+wide build {min(builds):8.2f} ms wall (device {s.build_ms:7.2f} ms; wide at first use "
              f"{wi['build_ms']:8.2f} ms) depth {wi['depth']} slots {wi['slots']}  frame {best.kernel_ms:8.2f} ms  "
              f"visits {best.node_visits} tris {best.tri_tests} rays {best.rays}", flush=True)
    first = next(iter(out.values()))
    same = all(np.array_equal(first.view(np.uint32), o.view(np.uint32)) for o in out.values())
    print(f"{cfg} frames identical: {same}", flush=True)
