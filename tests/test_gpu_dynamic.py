"""GPU tests: dynamic scenes -- objects updated in place and the LBVH rebuilt on the device every
frame ("per-frame rebuild for dynamic scenes").

The reference builds its BVH once per run (main.cu:122-128, bvh.h:132-145); a moving scene there
means a new world.  Here pt_scene_update_objects + pt_scene_build_bvh rebuild in place, reusing
every device buffer.  The checker: a rebuilt scene equals, node for node and pixel for pixel, a
scene created from scratch with the same objects, and the oracle's LBVH of those objects.
Bar: bit-exact.
"""
import numpy as np
import pytest

from helpers import random_rays, random_soup, rays_to_struct

pytestmark = pytest.mark.gpu

W, H = 48, 32


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assert_nodes_equal(g, o):
    for f in ("left", "right", "parent", "objid"):
        np.testing.assert_array_equal(g[f], o[f], err_msg=f)
    np.testing.assert_array_equal(bits(g["bmin"]), bits(o["bmin"]))
    np.testing.assert_array_equal(bits(g["bmax"]), bits(o["bmax"]))


def moved(pt, objs, frame, rng):
    """Frame `frame` of a simple animation: every object drifts by its own offset."""
    out = objs.copy()
    off = (rng.normal(size=(len(objs), 3)) * 0.05 * frame).astype(np.float32)
    sph = out["type"] == pt.PT_SPHERE
    out["v"][sph, 0:3] += off[sph]
    for k in range(3):
        out["v"][~sph, 3 * k:3 * k + 3] += off[~sph]
    return out


@pytest.mark.parametrize("name", ["rtiow", "bunny_cornell"])
def test_rebuild_matches_fresh_scene(pt, orc, gpu, name):
    p = pt.Preset(name, W, H)
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    for frame in (1, 2, 3):
        objs = moved(pt, p.objects, frame, np.random.default_rng(3))
        scene.update_objects(objs)
        scene.build_bvh()
        fresh = pt.Scene(objs, p.materials, device=gpu)
        got = scene.download_bvh()
        assert_nodes_equal(got, fresh.download_bvh())
        assert_nodes_equal(got, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True))
        assert scene.bvh_info() == fresh.bvh_info()
        for r in (pt.RNG_COMPAT, pt.RNG_SAMPLE):
            a, _ = pt.render(scene, pt.Film(W, H, seed=frame), p.camera, 2, 50, rng=r)
            b, _ = pt.render(fresh, pt.Film(W, H, seed=frame), p.camera, 2, 50, rng=r)
            np.testing.assert_array_equal(bits(a), bits(b))


def test_partial_update_and_oracle_frame(pt, orc, gpu):
    """Update a range of objects only; the frame equals the oracle's render of the new scene."""
    objs, mats = random_soup(300, 40, seed=21, spread=8.0)
    scene = pt.Scene(objs, mats, device=gpu)
    new = objs.copy()
    new[100:180] = moved(pt, objs[100:180], 4, np.random.default_rng(9))
    scene.update_objects(new[100:180], first=100)
    np.testing.assert_array_equal(scene.objects, new)
    scene.build_bvh()
    nodes = orc.build_lbvh(new, orc.morton_keys(new), tight=True)
    assert_nodes_equal(scene.download_bvh(), nodes)
    cam = pt.camera_make((0, 2, 20), (0, 0, 0), 40.0, W / H)
    film = pt.Film(W, H, seed=5)
    rgb, _ = pt.render(scene, film, cam, 2, 8)
    want, _, _ = orc.render_sums(new, mats, nodes, pt.camera_to_array(cam), W, H, film.rows, 2, 8,
                                 orc.film_states(5, W, film.rows), nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(want))


def test_stale_bvh_rejected(pt, gpu):
    p = pt.Preset("rtiow", W, H)
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    scene.update_objects(p.objects[:3])
    with pytest.raises(pt.PtError):
        pt.render(scene, pt.Film(W, H, seed=1), p.camera, 1, 4)
    rays = np.zeros(4, pt.RAY_DTYPE)
    rays["d"] = (0, 0, -1)
    with pytest.raises(pt.PtError):
        scene.trace(rays)
    scene.build_bvh()
    pt.render(scene, pt.Film(W, H, seed=1), p.camera, 1, 4)


def test_update_validation(pt, gpu):
    p = pt.Preset("rtiow", W, H)
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    n = len(p.objects)
    bad_mat = p.objects[:2].copy()
    bad_mat["mat"][1] = len(p.materials)
    bad_type = p.objects[:2].copy()
    bad_type["type"][0] = 2
    for objs, first in ((p.objects[:2], n - 1), (p.objects[:2], -1), (bad_mat, 0), (bad_type, 0)):
        with pytest.raises(pt.PtError):
            scene.update_objects(objs, first=first)
    # a rejected update leaves the scene untouched and built
    film = pt.Film(W, H, seed=2)
    a, _ = pt.render(scene, film, p.camera, 1, 8)
    b, _ = pt.render(pt.Scene(p.objects, p.materials, device=gpu), pt.Film(W, H, seed=2), p.camera, 1, 8)
    np.testing.assert_array_equal(bits(a), bits(b))


def test_c5_rebuild_per_frame(pt, gpu):
    """1,043,312 triangles moved and rebuilt three times: the rebuild reuses the first build's
    buffers and stays within a frame budget (device time; printed for DESIGN.md)."""
    p = pt.Preset("bunny_field")
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    first = scene.build_ms
    times = []
    for frame in (1, 2, 3):
        objs = p.objects.copy()
        objs["v"] += np.float32(0.01 * frame)
        scene.update_objects(objs)
        scene.build_bvh()
        times.append(scene.build_ms)
    print(f"C5 build {first:.2f} ms, rebuilds {[round(t, 2) for t in times]} ms")
    assert scene.bvh_info()["nodes"] == 2 * len(p.objects) - 1
    assert max(times) < 50.0


@pytest.fixture(params=["sah", "ploc"])
def builder(request, monkeypatch):
    """The device wide tree's binary builder (PT_WIDE_DEVICE_BUILDER)."""
    monkeypatch.setenv("PT_WIDE_DEVICE_BUILDER", request.param)
    return request.param


def test_wide_device_rebuild_per_frame(pt, orc, gpu, builder):
    """Moving objects rendered with the wide kernel, its tree rebuilt on the device every frame
    (PT_BVH_WIDE_DEVICE): each frame equals the binary kernel's frame of a fresh scene and, for
    compat streams, the oracle's render; the rebuild is deterministic (same stats twice)."""
    flags = pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_WIDE_DEVICE
    objs0, mats = random_soup(600, 80, seed=31, spread=8.0)
    scene = pt.Scene(objs0, mats, device=gpu, flags=flags)
    cam = pt.camera_make((0, 2, 20), (0, 0, 0), 40.0, W / H)
    for frame in (1, 2, 3):
        objs = moved(pt, objs0, frame, np.random.default_rng(40 + frame))
        scene.update_objects(objs)
        scene.build_bvh(flags)
        assert scene.wide_info()["source"] == 2
        fresh = pt.Scene(objs, mats, device=gpu)
        a, sa = pt.render(scene, pt.Film(W, H, seed=frame), cam, 2, 10, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
        b, sb = pt.render(fresh, pt.Film(W, H, seed=frame), cam, 2, 10, kernel=pt.KERNEL_WAVEFRONT, rng=pt.RNG_SAMPLE)
        np.testing.assert_array_equal(bits(a), bits(b))
        assert sa.rays == sb.rays
        scene.build_bvh(flags)   # same objects again: the same tree
        a2, sa2 = pt.render(scene, pt.Film(W, H, seed=frame), cam, 2, 10, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
        np.testing.assert_array_equal(bits(a2), bits(a))
        assert (sa2.node_visits, sa2.tri_tests, sa2.sphere_tests) == (sa.node_visits, sa.tri_tests, sa.sphere_tests)
    film = pt.Film(W, H, seed=9)
    rgb, _ = pt.render(scene, film, cam, 2, 8, kernel=pt.KERNEL_WIDE)
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    want, _, _ = orc.render_sums(objs, mats, nodes, pt.camera_to_array(cam), W, H, film.rows, 2, 8,
                                 orc.film_states(9, W, film.rows), nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(want))


def test_wide_device_identical_objects(pt, orc, gpu, builder):
    """5,000 copies of one triangle and 3,000 of one sphere: every clustering distance ties (the
    pairing order must still halve the clusters each pass) and the reference's tie order decides
    every hit."""
    objs, mats = random_soup(1, 1, seed=50, n_mat=4)
    tri, sph = objs[:1], objs[1:2]
    assert tri["type"][0] == pt.PT_TRIANGLE and sph["type"][0] == pt.PT_SPHERE
    rep = np.concatenate([np.repeat(tri, 5000), np.repeat(sph, 3000)])
    rep["mat"] = np.arange(len(rep)) % 4
    flags = pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_WIDE_DEVICE
    scene = pt.Scene(rep, mats, device=gpu, flags=flags)
    info = scene.wide_info()
    assert info["source"] == 2 and 1 <= info["depth"] <= 8
    rays = random_rays(4096, seed=51, objects=rep)
    hits, _ = scene.trace(rays_to_struct(rays, pt.RAY_DTYPE), 0.001, np.inf, kernel=pt.KERNEL_WIDE)
    ref, _ = orc.trace(rep, orc.build_lbvh(rep, orc.morton_keys(rep), tight=True), rays, 0.001, np.inf)
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(hits[f], ref[f], err_msg=f)
    h = hits["hit"] == 1
    assert h.sum() > 100
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(bits(hits[f][h]), bits(ref[f][h]), err_msg=f)


def test_c5_wide_device_rebuild(pt, gpu, builder):
    """1,043,312 triangles: LBVH + device wide tree per frame within a frame budget; the frame
    equals the host-built wide tree's frame."""
    p = pt.Preset("bunny_field", 160, 90)
    flags = pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_WIDE_DEVICE
    scene = pt.Scene(p.objects, p.materials, device=gpu, flags=flags)
    times = []
    for frame in (1, 2):
        objs = p.objects.copy()
        objs["v"] += np.float32(0.01 * frame)
        scene.update_objects(objs)
        scene.build_bvh(flags)
        times.append(scene.build_ms)
    print(f"C5 LBVH + wide device ({builder}) rebuilds {[round(t, 2) for t in times]} ms, wide {scene.wide_info()}")
    assert max(times) < 100.0
    host = pt.Scene(objs, p.materials, device=gpu)
    a, _ = pt.render(scene, pt.Film(160, 90, seed=3), p.camera, 2, p.max_depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    b, _ = pt.render(host, pt.Film(160, 90, seed=3), p.camera, 2, p.max_depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    assert host.wide_info()["source"] == 1
    np.testing.assert_array_equal(bits(a), bits(b))


def test_updated_scene_builds_wide_tree_on_device(pt, gpu, monkeypatch):
    """A scene whose objects were updated is dynamic: without PT_BVH_WIDE_DEVICE its wide tree is
    still built on the device at first use (a host SAH build per frame would dominate); a static
    scene keeps the host tree.  The frames are the same either way."""
    monkeypatch.delenv("PT_WIDE_BUILD", raising=False)
    objs, mats = random_soup(400, 60, seed=61, spread=8.0)
    cam = pt.camera_make((0, 2, 20), (0, 0, 0), 40.0, W / H)
    static = pt.Scene(objs, mats, device=gpu)
    a, _ = pt.render(static, pt.Film(W, H, seed=2), cam, 2, 8, kernel=pt.KERNEL_WIDE)
    assert static.wide_info()["source"] == 1
    dyn = pt.Scene(objs, mats, device=gpu)
    dyn.update_objects(objs[:10])
    dyn.build_bvh()
    assert dyn.wide_info()["source"] == 0   # not built yet
    b, _ = pt.render(dyn, pt.Film(W, H, seed=2), cam, 2, 8, kernel=pt.KERNEL_WIDE)
    assert dyn.wide_info()["source"] == 2
    np.testing.assert_array_equal(bits(a), bits(b))
