"""Full-size frames at BASELINE.json's configurations (GPU only).

* C4 (configs[3]): the C3 scene at 1920x1080 and 4096 spp in the 8-GPU layout -- 8-row stripes,
  stripe s on part s % 8 -- rendered as 8 parts on one GPU.  Every pixel of a sample-mode frame
  is a function of (seed, pixel, sample) alone (the reference keys its streams by pixel,
  main.cu:262-269) and a pixel's block sums are added exactly, so the assembled frame must equal
  the one-part frame bit for bit; two of its rows are checked against the oracle at the full
  4096 spp, and the parts' ray counts must add up to the one-part frame's.
* The wide kernel's full frames against the reference-order kernel (binary LBVH, the reference's
  visiting order) at C2 (256 spp), C3 (64 spp) and C5 (16 spp): every pixel and the ray count equal.
"""
import numpy as np
import pytest
import torch  # noqa: F401  (before libpt.so loads: they share torch's HIP runtime)

pytestmark = pytest.mark.gpu

STRIPE = 8


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assemble(parts, h, w, n):
    """Frame rows from n stripe-partitioned films (stripe s -> part s % n), film order."""
    img = np.zeros((h, w, 3), np.float32)
    for k, (rows, rgb) in enumerate(parts):
        img[rows] = rgb.reshape(len(rows), w, 3)
    return img


def test_c4_eight_stripes_4096spp(pt, orc, gpu):
    p = pt.Preset("bunny_cornell")
    w, h, spp, depth, seed = p.width, p.height, 4096, p.max_depth, 1
    assert (w, h) == (1920, 1080)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    one = pt.Film(w, h, seed, device=gpu, stripe_height=STRIPE)
    full, fst = pt.render(s, one, p.camera, spp, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    parts, rays = [], 0
    for k in range(8):
        f = pt.Film(w, h, seed, device=gpu, stripe_height=STRIPE, n_parts=8, part=k)
        rgb, st = pt.render(s, f, p.camera, spp, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
        parts.append((f.rows.copy(), rgb))
        rays += st.rays
        f.close()
    img = assemble(parts, h, w, 8)
    assert np.array_equal(bits(img.reshape(-1, 3)), bits(full)), "8-part frame differs from the 1-part frame"
    assert rays == fst.rays and fst.paths == w * h * spp
    assert fst.rays > 4 * w * h * spp   # ~4.7 rays per path at depth 50
    # two rows against the oracle at the full sample count: one through the slow pixels under the
    # bunny, one through the upper box
    rows = np.array([90, 700], np.int32)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    ref, _ = orc.render_sample(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, rows, spp, depth,
                               seed, max(16, -(-spp // 64)), nthreads=16)
    got = full.reshape(h, w, 3)[rows].reshape(-1, 3)
    assert np.array_equal(bits(got), bits(ref)), "rows differ from the oracle at 4096 spp"


@pytest.mark.parametrize("name,spp,rng", [
    ("cornell", 256, "sample"),          # C2, full frame and sample count
    ("bunny_cornell", 64, "sample"),     # C3 at 1/16 of its sample count
    ("bunny_cornell", 8, "compat"),
    ("bunny_field", 16, "sample"),       # C5 at 1/32 of its sample count
])
def test_fullsize_wide_equals_reference_order(pt, gpu, name, spp, rng):
    p = pt.Preset(name)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    mode = pt.RNG_SAMPLE if rng == "sample" else pt.RNG_COMPAT
    out = {}
    for k in (pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
        f = pt.Film(p.width, p.height, 1, device=gpu)
        out[k] = pt.render(s, f, p.camera, spp, p.max_depth, kernel=k, rng=mode)
        f.close()
    (a, sa), (b, sb) = out[pt.KERNEL_WAVEFRONT], out[pt.KERNEL_WIDE]
    assert np.array_equal(bits(a), bits(b)), f"{int((bits(a) != bits(b)).any(1).sum())} pixels differ"
    assert sa.rays == sb.rays and sa.paths == sb.paths == p.width * p.height * spp
