"""Device SAH wide build on a few presets with a sync after every launch (PT_SAH_SYNC=1): names
the failing kernel.  Exits 3 on any failure so that a GPU step sequence stops there."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import torch  # noqa: E402,F401
import ptamd as pt  # noqa: E402

os.environ["PT_SAH_SYNC"] = "1"
os.environ.pop("PT_WIDE_DEVICE_BUILDER", None)
bad = 0
for name in sys.argv[1:] or ["triangle_world", "cornell", "bunny_cornell", "random_world"]:
    p = pt.Preset(name, 64, 64)
    try:
        s = pt.Scene(p.objects, p.materials, flags=pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_WIDE_DEVICE)
        print(name, len(p.objects), "ok", s.wide_info(), flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, len(p.objects), "FAIL", e, flush=True)
        bad = 1
        break
sys.exit(3 if bad else 0)
