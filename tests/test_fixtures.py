"""The committed oracle fixtures (tests/golden/oracle_fixtures.npz, SURVEY.md §8(c) F1-F5, made
by tools/make_fixtures.py) against the CPU restatement and the library's host builders: every
array bit for bit.  A change to the oracle, the scene presets or the host Morton keys that moves
any output fails here; the GPU counterpart is tests/test_gpu_fixtures.py."""
import os

import numpy as np
import pytest

from helpers import read_png

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(REPO, "tests", "golden", "oracle_fixtures.npz")


@pytest.fixture(scope="module")
def fx():
    with np.load(FIX) as d:   # plain arrays only (allow_pickle stays False)
        return {k: d[k] for k in d.files}


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assert_nodes_equal(g, o):
    for f in ("left", "right", "parent", "objid"):
        np.testing.assert_array_equal(g[f], o[f], err_msg=f)
    np.testing.assert_array_equal(bits(g["bmin"]), bits(o["bmin"]))
    np.testing.assert_array_equal(bits(g["bmax"]), bits(o["bmax"]))


def assert_hits_equal(g, o):
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(g[f], o[f], err_msg=f)
    h = o["hit"] == 1
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(bits(g[f][h]), bits(o[f][h]), err_msg=f)


@pytest.mark.parametrize("key,name", [("c1", "rtiow"), ("tw", "triangle_world"), ("c2", "cornell"),
                                      ("c3", "bunny_cornell")])
def test_presets_build_the_fixture_scenes(pt, fx, key, name):
    """pt_preset_scene (host: OBJ loader, mt19937 scene layout, camera) reproduces the inputs."""
    w, h = (int(v) for v in fx[f"{key}_size"])
    p = pt.Preset(name, w if key != "tw" else 0, h if key != "tw" else 0)
    assert (p.width, p.height) == (w, h)
    np.testing.assert_array_equal(p.objects.view(np.uint8), fx[f"{key}_objects"].view(np.uint8))
    np.testing.assert_array_equal(p.materials.view(np.uint8), fx[f"{key}_materials"].view(np.uint8))
    np.testing.assert_array_equal(bits(pt.camera_to_array(p.camera)), bits(fx[f"{key}_camera"]))


@pytest.mark.parametrize("key", ["c2", "c3"])
def test_f1_morton_keys(pt, orc, fx, key):
    objs = fx[f"{key}_objects"]
    np.testing.assert_array_equal(orc.morton_keys(objs), fx[f"f1_{key}_keys"])
    np.testing.assert_array_equal(pt.morton_keys(objs), fx[f"f1_{key}_keys"])   # libpt's host keys
    k = fx[f"f1_{key}_keys"]
    assert (np.diff((k >> np.uint64(32)).astype(np.int64)) >= 0).all()   # sorted by code, stable in objID


@pytest.mark.parametrize("key", ["c2", "c3", "tw"])
def test_f2_lbvh(orc, fx, key):
    objs = fx[f"{key}_objects"]
    keys = orc.morton_keys(objs)
    assert_nodes_equal(orc.build_lbvh(objs, keys, tight=True), fx[f"f2_{key}_tight"])
    if f"f2_{key}_ref" in fx:   # the reference's origin-inflated boxes (bvh.h:117-130)
        ref = fx[f"f2_{key}_ref"]
        assert_nodes_equal(orc.build_lbvh(objs, keys, tight=False), ref)
        # same topology as the tight tree; every internal box contains the origin
        for f in ("left", "right", "parent", "objid"):
            np.testing.assert_array_equal(ref[f], fx[f"f2_{key}_tight"][f])
        n = len(objs)
        assert (ref["bmin"][:n - 1] <= 0).all() and (ref["bmax"][:n - 1] >= 0).all()


@pytest.mark.parametrize("key", ["c2", "c3", "tw"])
def test_f3_closest_hits(orc, fx, key):
    objs, rays = fx[f"{key}_objects"], fx[f"f3_{key}_rays"]
    hits, st = orc.trace(objs, fx[f"f2_{key}_tight"], rays)
    assert_hits_equal(hits, fx[f"f3_{key}_hits"])
    assert [st.node_visits, st.tri_tests, st.sphere_tests] == list(fx[f"f3_{key}_counts"])
    brute, _ = orc.trace(objs, None, rays, brute=True)   # RenderManager::hit (render_manager.h:71-84)
    assert_hits_equal(brute, fx[f"f3_{key}_hits"])


def test_f4_scatter_tapes(orc, fx):
    rays, hits, mats = fx["f3_c3_rays"], fx["f3_c3_hits"], fx["f4_materials"]
    assert sorted(set(fx["f4_mat"].tolist())) == [0, 1, 2]
    for j in range(len(fx["f4_mat"])):
        m, i = int(fx["f4_mat"][j]), int(fx["f4_case"][j])
        ok, out, att, used = orc.scatter_tape(mats[m], rays[i], hits[i], fx["f4_tape"][j])
        assert int(ok) == fx["f4_ok"][j] and used == fx["f4_used"][j]
        np.testing.assert_array_equal(bits(out), bits(fx["f4_out"][j]))
        np.testing.assert_array_equal(bits(att), bits(fx["f4_att"][j]))
    # the Lambertian rejection loop consumes 3 draws per trial
    assert (fx["f4_used"][fx["f4_mat"] == 0] % 3 == 0).all()


@pytest.mark.parametrize("key", ["c1", "c2"])
def test_f5_compat_frames(orc, fx, key):
    objs, mats, cam = fx[f"{key}_objects"], fx[f"{key}_materials"], fx[f"{key}_camera"]
    w, h = (int(v) for v in fx[f"{key}_size"])
    spp, depth, seed = (int(v) for v in fx[f"f5_{key}_params"])
    rows = np.arange(h, dtype=np.int32)
    states = orc.film_states(seed, w, rows)
    rgb, st = orc.render(objs, mats, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), cam, w, h, rows, spp,
                         depth, states, nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(fx[f"f5_{key}_rgb"]))
    assert [st.rays, st.paths] == list(fx[f"f5_{key}_counts"])
    if f"f5_{key}_rng_after" in fx:
        np.testing.assert_array_equal(states, fx[f"f5_{key}_rng_after"])


def test_f5_c1_png_bytes(pt, orc, fx, tmp_path):
    """saveColor on the fixture frame: the oracle's quantiser, libpt's and the written PNG agree."""
    w, h = (int(v) for v in fx["c1_size"])
    q = fx["f5_c1_rgba8"]
    np.testing.assert_array_equal(orc.quantize_png(fx["f5_c1_rgb"]), q)
    flipped = q.reshape(h, w, 4)[::-1]   # PngImage rows: top first (main.cu:481)
    np.testing.assert_array_equal(pt.quantize_rgba8(fx["f5_c1_rgb"], w, h).reshape(h, w, 4), flipped)
    path = str(tmp_path / "c1.png")
    pt.write_png(path, fx["f5_c1_rgb"], w, h)
    np.testing.assert_array_equal(read_png(path), flipped)


def test_f5_c3_sample_mode_frame(orc, fx):
    objs, mats, cam = fx["c3_objects"], fx["c3_materials"], fx["c3_camera"]
    w, h = (int(v) for v in fx["c3_size"])
    spp, depth, seed, chunk = (int(v) for v in fx["f5_c3_sample_params"])
    rgb, st = orc.render_sample(objs, mats, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), cam, w, h,
                                np.arange(h, dtype=np.int32), spp, depth, seed, chunk, nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(fx["f5_c3_sample_rgb"]))
    assert [st.rays, st.paths] == list(fx["f5_c3_sample_counts"])
