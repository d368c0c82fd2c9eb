"""Thin-lens cameras (camera::get_ray, camera.h:58-62: aperture > 0, defocus blur).

The reference draws the lens sample from the shared randState[0] (main.cu:286), a race between
all threads, so its defocused frames are not reproducible; ours draw it from the path's own stream
after the pixel jitter.  The oracle restates exactly that, so every kernel and both
RNG modes must equal it bit for bit.  The statistical pin against the reference's own defocused
render (output/11.png) is tests/test_oracle.py::test_reference_chapter_renders.
"""
import numpy as np
import pytest
import torch  # before libpt.so loads (the two must share torch's HIP runtime)

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("name,aperture", [("rtiow", 0.1), ("rtiow", 2.0), ("bunny_cornell", 40.0)])
def test_defocus_frames_match_oracle(pt, orc, gpu, name, aperture):
    p = pt.Preset(name, 96, 54)
    w, h = p.width, p.height
    c = pt.camera_to_array(p.camera)
    frm, front = c[0:3], c[18:21]
    focus = 10.0 if name == "rtiow" else 800.0
    cam = pt.camera_make(frm, frm - front, 20.0 if name == "rtiow" else 40.0, w / h, aperture, focus)
    assert cam.lens_radius == np.float32(aperture / 2)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    depth = min(p.max_depth, 12)
    rows = np.arange(h, dtype=np.int32)
    ref_c, rst_c = orc.render(p.objects, p.materials, nodes, pt.camera_to_array(cam), w, h, rows, 3, depth,
                              orc.film_states(5, w, rows), nthreads=8)
    ref_s, rst_s = orc.render_sample(p.objects, p.materials, nodes, pt.camera_to_array(cam), w, h, rows, 3, depth, 5, 2,
                                     nthreads=8)
    for k in (pt.KERNEL_SIMPLE, pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
        rgb, st = pt.render(s, pt.Film(w, h, 5, device=gpu), cam, 3, depth, kernel=k)
        np.testing.assert_array_equal(bits(rgb), bits(ref_c), err_msg=f"compat kernel {k}")
        assert st.rays == rst_c.rays
        rgb, st = pt.render(s, pt.Film(w, h, 5, device=gpu), cam, 3, depth, kernel=k, rng=pt.RNG_SAMPLE, chunk=2)
        np.testing.assert_array_equal(bits(rgb), bits(ref_s), err_msg=f"sample kernel {k}")
        assert st.rays == rst_s.rays
    # a lens changes the frame (the pinhole frame differs), and blurs: lower mean gradient
    pin, _ = pt.render(s, pt.Film(w, h, 5, device=gpu), p.camera if name != "rtiow" else
                       pt.camera_make(frm, frm - front, 20.0, w / h, 0.0, focus), 3, depth, rng=pt.RNG_SAMPLE, chunk=2)
    assert not np.array_equal(bits(pin), bits(ref_s))


def test_lens_radius_validation(pt, gpu):
    p = pt.Preset("cornell", 16, 16)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    cam = pt.Camera.from_buffer_copy(bytes(p.camera))
    for bad in (-1.0, float("nan"), float("inf")):
        cam.lens_radius = bad
        with pytest.raises(pt.PtError):
            pt.render(s, pt.Film(16, 16, 1, device=gpu), cam, 1, 4)
