"""Regenerate models/ from the reference's model data (run in the survey container only).

The reference ships the Stanford bunny and the Cornell-box geometry as OBJ files
(models/bunny/bunny.obj, models/cornellbox/*.obj).  They are benchmark INPUT DATA, not
source.  This script re-emits them as OBJ with every coordinate written as the shortest
decimal that round-trips to the same float32 (parsed with the C library's strtof, as the
reference's loader does via std::stof), so the triangles are bit-identical to what the
reference would load.  The GPU box has no /root/reference; it reads models/ from the repo.

usage: python tools/convert_models.py [/root/reference/models] [models]
"""
import ctypes
import os
import sys

import numpy as np

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def strtof(tok: str) -> np.float32:
    return np.float32(_libc.strtof(tok.encode(), None))


def fmt(x: np.float32) -> str:
    return np.format_float_positional(x, unique=True, trim="-")


def convert(src: str, dst: str) -> None:
    out = [f"# derived from the reference's {os.path.basename(src)} by tools/convert_models.py\n"]
    nv = nf = 0
    with open(src) as f:
        for line in f:
            parts = line.split()
            if not parts or parts[0].startswith("#"):
                continue
            if parts[0] in ("v", "vn", "vt"):
                vals = [strtof(t) for t in parts[1:]]
                for t, v in zip(parts[1:], vals):
                    assert strtof(fmt(v)) == v, (t, v)
                out.append(parts[0] + " " + " ".join(fmt(v) for v in vals) + "\n")
                nv += parts[0] == "v"
            elif parts[0] == "f":
                out.append("f " + " ".join(parts[1:]) + "\n")
                nf += 1
            else:
                out.append(" ".join(parts) + "\n")
    out.insert(1, f"# vertices {nv} faces {nf}\n")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        f.writelines(out)


def main() -> None:
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/models"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "models")
    for sub in ("bunny", "cornellbox"):
        for name in sorted(os.listdir(os.path.join(src, sub))):
            if name.endswith(".obj"):
                convert(os.path.join(src, sub, name), os.path.join(dst, sub, name))
                print("wrote", os.path.join(dst, sub, name))


if __name__ == "__main__":
    main()
