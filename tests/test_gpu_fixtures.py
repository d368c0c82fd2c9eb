"""The HIP path (through the C ABI) against the committed oracle fixtures
(tests/golden/oracle_fixtures.npz; tools/make_fixtures.py): device LBVH,
closest hits of both traversals, compat frames with their advanced RNG streams, the on-device
saveColor quantiser and a sample-mode frame.  Tolerance 0 ulp everywhere; these
tests need no oracle at run time."""
import os

import numpy as np
import pytest

from helpers import rays_to_struct

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(REPO, "tests", "golden", "oracle_fixtures.npz")


@pytest.fixture(scope="module")
def fx():
    with np.load(FIX) as d:
        return {k: d[k] for k in d.files}


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def camera(pt, arr):
    return pt.Camera.from_buffer_copy(np.ascontiguousarray(arr, np.float32).tobytes())


@pytest.mark.parametrize("key", ["c2", "c3", "tw"])
def test_device_lbvh_equals_fixture(pt, gpu, fx, key):
    s = pt.Scene(fx[f"{key}_objects"], fx[f"{key}_materials"], device=gpu)
    g, o = s.download_bvh(), fx[f"f2_{key}_tight"]
    for f in ("left", "right", "parent", "objid"):
        np.testing.assert_array_equal(g[f], o[f], err_msg=f)
    np.testing.assert_array_equal(bits(g["bmin"]), bits(o["bmin"]))
    np.testing.assert_array_equal(bits(g["bmax"]), bits(o["bmax"]))


@pytest.mark.parametrize("kernel", ["binary", "wide"])
@pytest.mark.parametrize("key", ["c2", "c3", "tw"])
def test_closest_hits_equal_fixture(pt, gpu, fx, key, kernel):
    s = pt.Scene(fx[f"{key}_objects"], fx[f"{key}_materials"], device=gpu)
    k = pt.KERNEL_WIDE if kernel == "wide" else pt.KERNEL_SIMPLE
    hits, st = s.trace(rays_to_struct(fx[f"f3_{key}_rays"], pt.RAY_DTYPE), kernel=k)
    o = fx[f"f3_{key}_hits"]
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(hits[f], o[f], err_msg=f)
    h = o["hit"] == 1
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(bits(hits[f][h]), bits(o[f][h]), err_msg=f)
    if kernel == "binary":   # the reference's visiting order: the same node visits and tests
        assert [st.node_visits, st.tri_tests, st.sphere_tests] == list(fx[f"f3_{key}_counts"])


@pytest.mark.parametrize("kernel", ["wide", "wavefront", "simple"])
@pytest.mark.parametrize("key", ["c1", "c2"])
def test_compat_frames_equal_fixture(pt, gpu, fx, key, kernel):
    w, h = (int(v) for v in fx[f"{key}_size"])
    spp, depth, seed = (int(v) for v in fx[f"f5_{key}_params"])
    s = pt.Scene(fx[f"{key}_objects"], fx[f"{key}_materials"], device=gpu)
    f = pt.Film(w, h, seed, device=gpu)
    k = {"wide": pt.KERNEL_WIDE, "wavefront": pt.KERNEL_WAVEFRONT, "simple": pt.KERNEL_SIMPLE}[kernel]
    rgb, st = pt.render(s, f, camera(pt, fx[f"{key}_camera"]), spp, depth, kernel=k)
    np.testing.assert_array_equal(bits(rgb), bits(fx[f"f5_{key}_rgb"]))
    assert [st.rays, st.paths] == list(fx[f"f5_{key}_counts"])
    if f"f5_{key}_rng_after" in fx:   # the film's XORWOW streams advanced exactly as the oracle's
        np.testing.assert_array_equal(f.get_rng(), fx[f"f5_{key}_rng_after"])


def test_device_quantised_frame_equals_fixture_png(pt, gpu, fx):
    w, h = (int(v) for v in fx["c1_size"])
    spp, depth, seed = (int(v) for v in fx["f5_c1_params"])
    s = pt.Scene(fx["c1_objects"], fx["c1_materials"], device=gpu)
    q, _ = pt.render(s, pt.Film(w, h, seed, device=gpu), camera(pt, fx["c1_camera"]), spp, depth,
                     out_format=pt.OUT_RGBA8)
    np.testing.assert_array_equal(q.reshape(-1, 4), fx["f5_c1_rgba8"])


@pytest.mark.parametrize("kernel", ["wide", "wavefront"])
def test_sample_mode_frame_equals_fixture(pt, gpu, fx, kernel):
    w, h = (int(v) for v in fx["c3_size"])
    spp, depth, seed, chunk = (int(v) for v in fx["f5_c3_sample_params"])
    s = pt.Scene(fx["c3_objects"], fx["c3_materials"], device=gpu)
    k = pt.KERNEL_WIDE if kernel == "wide" else pt.KERNEL_WAVEFRONT
    rgb, st = pt.render(s, pt.Film(w, h, seed, device=gpu), camera(pt, fx["c3_camera"]), spp, depth,
                        rng=pt.RNG_SAMPLE, chunk=chunk, kernel=k)
    np.testing.assert_array_equal(bits(rgb), bits(fx["f5_c3_sample_rgb"]))
    assert [st.rays, st.paths] == list(fx["f5_c3_sample_counts"])
