"""Generate tests/golden/ fixtures from the reference's committed data (survey container only).

exp2_blocks.npy — the reference's committed render output2/exp2.png (TRIANGLEWORLD, the
  reference's default scene, 1200x675, spp/seed unrecorded) reduced to 25x25-pixel block means
  in LINEAR radiance: each 8-bit value v was written as floor(clamp(sqrt(L),0,.999)*256)
  (png_image.h:24-30, main.cu:290-293), so L ~= ((v+0.5)/256)^2.  Block means of L are
  unbiased at any spp, which lets a low-spp oracle render be compared with it.  Rows are
  stored bottom-up (row 0 = bottom, the render kernel's order).

chapter_blocks.npz — the reference's committed chapter renders output/{8_sampleOnSphere, 8, 9, 10,
  11, 13, 13_1, 13_2}.png (the RTIOW chapter scenes the project was built through; their scene
  code is no longer in the repository, tests/test_oracle.py restates them) as the same linear
  block means.  13*.png are three renders of the final scene with different random small spheres:
  stored as their mean and the mask of "consensus" blocks where the three agree within 0.004
  (sky and the big spheres, untouched by the random spheres).

usage: python tools/make_golden.py [/root/reference]
"""
import os
import struct
import sys
import zlib

import numpy as np

BLOCK = 25


def read_png(path: str) -> np.ndarray:
    """Minimal decoder: 8-bit RGB/RGBA, non-interlaced (what stb_image_write produces)."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = ctype = None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if typ == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            assert depth == 8 and interlace == 0 and ctype in (2, 6)
        elif typ == b"IDAT":
            idat += body
        elif typ == b"IEND":
            break
    ch = 4 if ctype == 6 else 3
    raw = zlib.decompress(idat)
    stride = w * ch
    img = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        out = np.zeros(stride, np.int32)
        for x in range(stride):
            a = out[x - ch] if x >= ch else 0
            b = prev[x]
            c = prev[x - ch] if x >= ch else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) >> 1
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            out[x] = (line[x] + p) & 0xFF
        img[y] = out
        prev = out
    return img.reshape(h, w, ch)


def linear_blocks(img8: np.ndarray, block: int = BLOCK) -> np.ndarray:
    h, w = img8.shape[:2]
    lin = ((img8[..., :3].astype(np.float64) + 0.5) / 256.0) ** 2
    lin = lin[::-1]  # bottom-up
    return lin.reshape(h // block, block, w // block, block, 3).mean(axis=(1, 3)).astype(np.float32)


def main() -> None:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out_dir = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
    os.makedirs(out_dir, exist_ok=True)
    img = read_png(os.path.join(ref, "output2", "exp2.png"))
    assert img.shape[:2] == (675, 1200), img.shape
    blocks = linear_blocks(img)
    np.save(os.path.join(out_dir, "exp2_blocks.npy"), blocks)
    print("exp2_blocks.npy", blocks.shape, float(blocks.mean()))
    out = {}
    for name in ("8_sampleOnSphere", "8", "9", "10", "11"):
        img = read_png(os.path.join(ref, "output", name + ".png"))
        assert img.shape[:2] == (600, 1200), (name, img.shape)
        out["c" + name] = linear_blocks(img)
    finals = [linear_blocks(read_png(os.path.join(ref, "output", n + ".png"))) for n in ("13", "13_1", "13_2")]
    spread = np.max([np.abs(a - b) for a in finals for b in finals], axis=0).max(axis=2)
    out["c13_mean"] = (sum(finals) / 3).astype(np.float32)
    out["c13_consensus"] = spread < 0.004
    np.savez_compressed(os.path.join(out_dir, "chapter_blocks.npz"), **out)
    print("chapter_blocks.npz", {k: v.shape for k, v in out.items()}, int(out["c13_consensus"].sum()))


if __name__ == "__main__":
    main()
