"""Traversal stacks deeper than the LDS part of the sample-mode stack.

Sample mode on trees deeper than 32 levels keeps 32 stack entries per lane in LDS (8 KB per
wave, 5 waves per SIMD) and the deeper entries in a global per-lane buffer.  C5's tree is 40+
levels deep but its rays rarely stack more than 32 entries, so this scene (helpers.
deep_stack_scene) forces it: every box contains the camera, so every camera ray walks the whole
tree and stacks 34 entries.  The checker is the oracle; bar: bit-exact.
"""
import numpy as np
import pytest

from helpers import deep_stack_scene, max_stack

W, H = 8, 6


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def test_scene_stacks_more_than_32():
    import oracle as orc
    objs, _ = deep_stack_scene()
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    assert max_stack(nodes, len(objs)) > 32
    assert 32 < orc.bvh_depth(nodes, len(objs)) + 1 <= 48   # STACK 48: 32 in LDS, 16 in memory


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["wavefront", "wide", "simple"])
def test_deep_stack_sample_mode_bit_exact(pt, orc, gpu, kernel):
    objs, mats = deep_stack_scene()
    scene = pt.Scene(objs, mats, device=gpu)
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    assert scene.bvh_info()["depth"] == orc.bvh_depth(nodes, len(objs))
    cam = pt.camera_make((1024.0, 1024.0, 1024.0), (1024.0, 900.0, 0.0), 60.0, W / H)
    film = pt.Film(W, H, seed=3, device=gpu)
    k = {"wavefront": pt.KERNEL_WAVEFRONT, "wide": pt.KERNEL_WIDE, "simple": pt.KERNEL_SIMPLE}[kernel]
    rgb, st = pt.render(scene, film, cam, 3, 3, rng=pt.RNG_SAMPLE, chunk=2, kernel=k)
    ref, rst = orc.render_sample(objs, mats, nodes, pt.camera_to_array(cam), W, H, film.rows, 3, 3, 3, 2,
                                 nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    assert st.rays == rst.rays
    if kernel != "wide":   # every camera ray visits every internal node (all boxes contain the camera)
        assert st.node_visits >= W * H * 3 * (len(objs) - 1)


@pytest.mark.gpu
def test_deep_stack_compat_bit_exact(pt, orc, gpu):
    objs, mats = deep_stack_scene()
    scene = pt.Scene(objs, mats, device=gpu)
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    cam = pt.camera_make((1024.0, 1024.0, 1024.0), (0.0, 1024.0, 1024.0), 60.0, W / H)
    film = pt.Film(W, H, seed=4, device=gpu)
    rgb, _ = pt.render(scene, film, cam, 2, 3)
    ref, _ = orc.render(objs, mats, nodes, pt.camera_to_array(cam), W, H, film.rows, 2, 3,
                        orc.film_states(4, W, film.rows), nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
