"""The compressed 8-wide tree (PT_KERNEL_WIDE) against the oracle's reference-order traversal.

The wide tree visits nodes in its own order (nearest child first) through conservative,
8-bit quantised boxes; the closest hit is the minimum of (t, the reference's tie order), which is
the hit the reference's left-first DFS keeps.  The bar is therefore the same as for the binary
kernels: every hit record bit-exact, including exact ties (duplicated triangles and spheres).
Every test runs on three trees: built on the host (binned SAH, at first use) and built on the
device by pt_scene_build_bvh (PT_BVH_WIDE_DEVICE: binned SAH, or PLOC with
PT_WIDE_DEVICE_BUILDER=ploc, then the collapse).
"""
import numpy as np
import pytest
import torch  # before libpt.so loads (the two must share torch's HIP runtime)

from helpers import OBJECT_DTYPE, MATERIAL_DTYPE, deep_stack_scene, random_rays, random_soup, rays_to_struct

pytestmark = pytest.mark.gpu

SCENES = ["triangle_world", "random_world", "test_world", "rtiow", "cornell", "bunny_cornell"]


@pytest.fixture(params=["host", "device", "device_ploc"])
def wb(request, monkeypatch):
    if request.param == "device_ploc":
        monkeypatch.setenv("PT_WIDE_DEVICE_BUILDER", "ploc")
    else:
        monkeypatch.delenv("PT_WIDE_DEVICE_BUILDER", raising=False)
    return request.param


def make_scene(pt, objs, mats, gpu, wb):
    flags = pt.PT_BVH_ORIGIN_BOUNDS | (pt.PT_BVH_WIDE_DEVICE if wb != "host" else 0)
    s = pt.Scene(objs, mats, device=gpu, flags=flags)
    if wb != "host" and len(objs):
        assert s.wide_info()["source"] == 2
    return s


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assert_hits_equal(g, o):
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(g[f], o[f], err_msg=f)
    h = g["hit"] == 1
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(bits(g[f][h]), bits(o[f][h]), err_msg=f)


def trace_both(pt, orc, gpu, wb, objs, mats, rays, tmin=0.001, tmax=np.inf):
    s = make_scene(pt, objs, mats, gpu, wb)
    hits, st = s.trace(rays_to_struct(rays, pt.RAY_DTYPE), tmin, tmax, kernel=pt.KERNEL_WIDE)
    assert s.wide_info()["source"] == (2 if wb != "host" else 1)
    ref, rst = orc.trace(objs, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), rays, tmin, tmax)
    return hits, st, ref, rst


@pytest.mark.parametrize("name", SCENES)
def test_wide_trace_matches_oracle(pt, orc, gpu, wb, name):
    p = pt.Preset(name)
    lo = p.objects["v"][:, :3].min(0)
    hi = p.objects["v"][:, :3].max(0)
    center = np.clip((lo + hi) / 2, -1e3, 1e3)
    radius = float(min(np.linalg.norm(hi - lo), 3000.0)) * 0.75 + 1.0
    rays = random_rays(8192, seed=2, center=center, radius=radius, objects=p.objects)
    hits, st, ref, rst = trace_both(pt, orc, gpu, wb, p.objects, p.materials, rays)
    assert_hits_equal(hits, ref)
    assert hits["hit"].sum() > 100
    assert st.rays == len(rays)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wide_trace_random_soup(pt, orc, gpu, wb, seed):
    objs, mats = random_soup(3000, 500, seed=seed)
    rays = random_rays(8192, seed=seed + 10, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)


def test_wide_trace_tmin_tmax_window(pt, orc, gpu, wb):
    objs, mats = random_soup(500, 100, seed=3)
    rays = random_rays(2048, seed=4, objects=objs)
    for tmin, tmax in ((0.001, 5.0), (2.0, 40.0), (0.0, np.inf)):
        hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays, tmin, tmax)
        assert_hits_equal(hits, ref)


def tie_scene(seed=5):
    """Exact ties: every triangle three times and every sphere three times (identical geometry,
    different materials), so the reference's order decides which copy is the hit: the FIRST
    triangle in key order (a later t == closest is rejected), the LAST sphere (t <= closest)."""
    objs, mats = random_soup(400, 120, seed=seed, n_mat=6)
    rep = np.concatenate([objs, objs, objs])
    rep["mat"][len(objs):2 * len(objs)] = (objs["mat"] + 1) % 6
    rep["mat"][2 * len(objs):] = (objs["mat"] + 2) % 6
    perm = np.random.default_rng(seed).permutation(len(rep))
    return rep[perm], mats


def test_wide_trace_exact_ties(pt, orc, gpu, wb):
    objs, mats = tie_scene()
    rays = random_rays(8192, seed=6, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)
    # the ties matter: the copies differ in material, and many rays hit a duplicated object
    assert (ref["hit"] == 1).sum() > 2000


def test_wide_trace_coplanar_sphere_ties(pt, orc, gpu, wb):
    """Concentric spheres of equal radius (the deep-stack scene: 2,048 identical spheres)."""
    objs, mats = deep_stack_scene(n_group=256)
    objs["mat"] = np.arange(len(objs)) % 1
    rays = random_rays(4096, seed=8, center=(1024.0, 1024.0, 1024.0), radius=3000.0, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)


def test_wide_trace_c5(pt, orc, gpu, wb):
    p = pt.Preset("bunny_field", 64, 36)
    rays = random_rays(8192, seed=9, center=(278, 150, 280), radius=700, objects=p.objects)
    hits, st, ref, rst = trace_both(pt, orc, gpu, wb, p.objects, p.materials, rays)
    assert_hits_equal(hits, ref)
    assert st.node_visits < rst.node_visits   # the point of the wide tree


@pytest.mark.parametrize("n", [1, 2, 3, 4, 9])
def test_wide_tiny_scenes(pt, orc, gpu, wb, n):
    """Roots that are a leaf (n <= 3) or a single wide node."""
    objs, mats = random_soup(n - n // 2, n // 2, seed=n)
    rays = random_rays(2048, seed=n, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)


def test_wide_render_ties_bit_exact(pt, orc, gpu, wb):
    """A rendered frame of the tie scene: every bounce's hit must be the reference's copy."""
    objs, mats = tie_scene(seed=11)
    w, h = 48, 32
    cam = pt.camera_make((0.0, 0.0, 30.0), (0.0, 0.0, 0.0), 50.0, w / h)
    s = make_scene(pt, objs, mats, gpu, wb)
    f = pt.Film(w, h, 5, device=gpu)
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    for rng in ("compat", "sample"):
        f.reset()
        if rng == "compat":
            rgb, st = pt.render(s, f, cam, 3, 12, kernel=pt.KERNEL_WIDE)
            ref, rst = orc.render(objs, mats, nodes, pt.camera_to_array(cam), w, h, f.rows, 3, 12,
                                  orc.film_states(5, w, f.rows), nthreads=8)
        else:
            rgb, st = pt.render(s, f, cam, 3, 12, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE, chunk=2)
            ref, rst = orc.render_sample(objs, mats, nodes, pt.camera_to_array(cam), w, h, f.rows, 3, 12, 5, 2,
                                         nthreads=8)
        np.testing.assert_array_equal(bits(rgb), bits(ref), err_msg=rng)
        assert st.rays == rst.rays


@pytest.mark.parametrize("cfg,w,h,spp", [("bunny_cornell", 240, 135, 4), ("bunny_field", 160, 90, 2), ("cornell", 128, 128, 8)])
def test_wide_frame_equals_reference_order_frame(pt, gpu, wb, cfg, w, h, spp):
    """Whole frames (both RNG modes) from the wide kernel equal the binary kernel's, which follows
    the reference's own visiting order (itself bit-exact against the oracle, test_gpu_parity.py)."""
    p = pt.Preset(cfg, w, h)
    s = make_scene(pt, p.objects, p.materials, gpu, wb)
    for rng in (pt.RNG_COMPAT, pt.RNG_SAMPLE):
        out = {}
        for k in (pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
            f = pt.Film(w, h, 7, device=gpu)
            out[k] = pt.render(s, f, p.camera, spp, p.max_depth, kernel=k, rng=rng)
        np.testing.assert_array_equal(bits(out[pt.KERNEL_WIDE][0]), bits(out[pt.KERNEL_WAVEFRONT][0]))
        assert out[pt.KERNEL_WIDE][1].rays == out[pt.KERNEL_WAVEFRONT][1].rays


@pytest.mark.parametrize("cfg,w,h,spp", [("bunny_cornell", 192, 108, 8), ("bunny_field", 160, 90, 2)])
def test_plane_margin_changes_work_not_frames(pt, gpu, monkeypatch, cfg, w, h, spp):
    """Round 6 (DESIGN §5 "Plane margin"): the host tree's child planes lie the tree's smallest
    quantum outside the exact boxes instead of one node quantum (PT_WIDE_MARGIN=0).  The margin is
    a pure performance choice: both RNG modes' frames stay bit-identical (and equal to the binary
    reference-order kernel's) while the tighter boxes visit fewer nodes and test fewer primitives."""
    p = pt.Preset(cfg, w, h)
    work = {}
    for margin in ("0", "1"):
        monkeypatch.setenv("PT_WIDE_MARGIN", margin)
        s = pt.Scene(p.objects, p.materials, device=gpu, flags=pt.PT_BVH_ORIGIN_BOUNDS)
        for rng in (pt.RNG_COMPAT, pt.RNG_SAMPLE):
            f = pt.Film(w, h, 7, device=gpu)
            work[margin, rng] = pt.render(s, f, p.camera, spp, p.max_depth, kernel=pt.KERNEL_WIDE, rng=rng)
        assert s.wide_info()["source"] == 1
    ref = pt.Scene(p.objects, p.materials, device=gpu, flags=pt.PT_BVH_ORIGIN_BOUNDS)
    for rng in (pt.RNG_COMPAT, pt.RNG_SAMPLE):
        (img0, st0), (img1, st1) = work["0", rng], work["1", rng]
        base = pt.render(ref, pt.Film(w, h, 7, device=gpu), p.camera, spp, p.max_depth, kernel=pt.KERNEL_WAVEFRONT,
                         rng=rng)[0]
        np.testing.assert_array_equal(bits(img1), bits(img0))
        np.testing.assert_array_equal(bits(img1), bits(base))
        assert st1.rays == st0.rays
        assert st1.node_visits < st0.node_visits and st1.tri_tests <= st0.tri_tests, (rng, st0, st1)


def test_wide_large_soup_trace_and_render(pt, orc, gpu, wb):
    """200,000 random triangles and spheres: hit records against the oracle, and a frame against
    the reference-order kernel."""
    objs, mats = random_soup(150_000, 50_000, seed=12, spread=60.0)
    rays = random_rays(8192, seed=13, radius=90.0, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)
    s = make_scene(pt, objs, mats, gpu, wb)
    cam = pt.camera_make((0.0, 20.0, 120.0), (0.0, 0.0, 0.0), 45.0, 1.5)
    frames = []
    for k in (pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
        f = pt.Film(96, 64, 3, device=gpu)
        frames.append(pt.render(s, f, cam, 2, 12, kernel=k, rng=pt.RNG_SAMPLE, chunk=2)[0])
    np.testing.assert_array_equal(bits(frames[1]), bits(frames[0]))


@pytest.mark.parametrize("name", ["bunny_cornell", "cornell"])
def test_device_sah_tree_quality(pt, gpu, monkeypatch, name):
    """The device's top-down SAH tree (PT_WIDE_DEVICE_BUILDER=sah) traverses like the host SAH
    tree: over the same rays its wide-node visits and primitive tests stay within 10 % of the
    host tree's (a wrong scan or sweep would still give valid trees and identical hits, only
    slower ones -- PLOC's tree, for scale, visits 7-10 % more nodes on these scenes)."""
    p = pt.Preset(name, 160, 90)
    rays = rays_to_struct(random_rays(20000, seed=91, objects=p.objects), pt.RAY_DTYPE)
    stats = {}
    for wb in ("host", "sah"):
        monkeypatch.setenv("PT_WIDE_DEVICE_BUILDER", "sah")
        flags = pt.PT_BVH_ORIGIN_BOUNDS | (pt.PT_BVH_WIDE_DEVICE if wb == "sah" else 0)
        s = pt.Scene(p.objects, p.materials, device=gpu, flags=flags)
        _, st = s.trace(rays, 0.001, np.inf, kernel=pt.KERNEL_WIDE)
        assert s.wide_info()["source"] == (2 if wb == "sah" else 1)
        stats[wb] = st
    h, d = stats["host"], stats["sah"]
    print(f"{name}: host visits {h.node_visits} tests {h.tri_tests + h.sphere_tests}; "
          f"device SAH visits {d.node_visits} tests {d.tri_tests + d.sphere_tests}")
    assert d.node_visits <= 1.10 * h.node_visits
    assert d.tri_tests + d.sphere_tests <= 1.10 * (h.tri_tests + h.sphere_tests)


def edge_scene(kind):
    """Scenes at the edges of the wide tree's encoding: tiny and huge coordinates (the plane
    quantum is relative to the scene extent), degenerate triangles, everything at one point, a
    huge ground sphere under small objects, very thin long triangles."""
    rng = np.random.default_rng(76)
    if kind == "tiny":
        objs, mats = random_soup(800, 200, seed=71, spread=10.0)
        objs["v"] *= np.float32(1e-3)
        return objs, mats, 0.02
    if kind == "huge":
        objs, mats = random_soup(800, 200, seed=72, spread=10.0)
        objs["v"] *= np.float32(1e4)
        objs["v"] += np.float32(3e5)
        return objs, mats, 2e5
    if kind == "degenerate":
        objs, mats = random_soup(600, 50, seed=73)
        tri = np.flatnonzero(objs["type"] == 3)
        objs["v"][tri[:200], 3:6] = objs["v"][tri[:200], 0:3]                 # zero-area: v1 == v0
        objs["v"][tri[200:300], 6:9] = 2 * objs["v"][tri[200:300], 3:6] - objs["v"][tri[200:300], 0:3]  # collinear
        return objs, mats, 15.0
    if kind == "one_point":
        objs, mats = random_soup(300, 100, seed=74, spread=0.0)
        objs["v"][objs["type"] == 1, :3] = 0.0
        return objs, mats, 5.0
    if kind == "ground":
        objs, mats = random_soup(500, 100, seed=75, spread=5.0)
        g = objs[-1:].copy()
        g["type"] = 1
        g["v"][0, :4] = (0.0, -1000.0, 0.0, 1000.0)
        return np.concatenate([objs, g]), mats, 20.0
    if kind == "slivers":
        n = 2000
        objs = np.zeros(n, OBJECT_DTYPE)
        objs["type"] = 3
        a = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
        axis = rng.integers(0, 3, n)
        b = a.copy()
        b[np.arange(n), axis] += np.float32(40.0)
        objs["v"][:, 0:3] = a
        objs["v"][:, 3:6] = b
        objs["v"][:, 6:9] = a + rng.uniform(-1e-3, 1e-3, (n, 3)).astype(np.float32)
        mats = np.zeros(2, MATERIAL_DTYPE)
        mats["type"] = 0
        mats["albedo"] = 0.5
        return objs, mats, 40.0
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["tiny", "huge", "degenerate", "one_point", "ground", "slivers"])
def test_wide_edge_scenes(pt, orc, gpu, wb, kind):
    objs, mats, radius = edge_scene(kind)
    lo = objs["v"][:, :3].min(0)
    hi = objs["v"][:, :3].max(0)
    center = (lo + hi) / 2 if kind != "ground" else np.zeros(3)
    rays = random_rays(4096, seed=80, center=center, radius=radius, objects=objs)
    hits, _, ref, _ = trace_both(pt, orc, gpu, wb, objs, mats, rays)
    assert_hits_equal(hits, ref)


def test_trace_device_pointers_match_host_api(pt, orc, gpu, wb):
    """pt_trace_closest_device on torch-owned device memory gives the host API's hit records, for
    both trees and the binary kernel."""
    objs, mats = random_soup(2000, 300, seed=91)
    rays = rays_to_struct(random_rays(5000, seed=92, objects=objs), pt.RAY_DTYPE)
    s = make_scene(pt, objs, mats, gpu, wb)
    dev = torch.device("cuda", gpu)
    rd = torch.from_numpy(rays.view(np.uint8).copy()).to(dev)
    for k in (pt.KERNEL_WIDE, pt.KERNEL_WAVEFRONT):
        want, wst = s.trace(rays, 0.001, np.inf, kernel=k)
        hd = torch.zeros(len(rays) * pt.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        st = s.trace_device(rd.data_ptr(), len(rays), hd.data_ptr(), 0.001, np.inf, kernel=k,
                            stream=torch.cuda.current_stream(dev).cuda_stream)
        got = hd.cpu().numpy().view(pt.HIT_DTYPE)
        assert_hits_equal(got, want)
        assert (st.rays, st.node_visits, st.tri_tests) == (wst.rays, wst.node_visits, wst.tri_tests)


@pytest.mark.parametrize("dist", [3.0, 7.5, 100.0, 1000.0])
def test_wide_trace_far_origins(pt, orc, gpu, wb, dist):
    """the wide boxes' one-quantum margin covers the rounding of the plane distances
    only for origins within about 11 scene extents; origins beyond 8 extents from the scene's
    centre are traced in the reference's order (wideFar).  Rays from `dist` extents away, aimed at
    the scene's primitives (many graze edges and corners of small nodes), must keep the
    reference's hits either way."""
    p = pt.Preset("bunny_cornell", 64, 36)
    objs = p.objects
    lo = objs["v"][:, :3].min(0)
    hi = objs["v"][:, :3].max(0)
    ext = float((hi - lo).max())
    rays = random_rays(8192, seed=int(dist) + 21, center=(lo + hi) / 2, radius=dist * ext, objects=objs)
    # aim half of the rays at triangle vertices and edge midpoints: grazing hits on tiny boxes
    rng = np.random.default_rng(int(dist))
    k = rng.integers(0, len(objs), 4096)
    v = objs["v"][k].reshape(-1, 3, 3)
    j = rng.integers(0, 3, 4096)
    tgt = np.where((np.arange(4096) % 2 == 0)[:, None], v[np.arange(4096), j],
                   0.5 * (v[np.arange(4096), j] + v[np.arange(4096), (j + 1) % 3]))
    rays[4096:, 3:] = (tgt - rays[4096:, :3]).astype(np.float32)
    hits, st, ref, rst = trace_both(pt, orc, gpu, wb, objs, p.materials, rays)
    assert_hits_equal(hits, ref)
    assert ref["hit"].sum() > 4000
    assert st.rays == len(rays)


def test_wide_render_far_camera(pt, orc, gpu, wb):
    """A camera 20 scene extents from the Cornell box (narrow field of view): its camera rays take
    the reference-order path, the bounces inside the box the wide tree; frame bit-exact."""
    p = pt.Preset("cornell", 48, 48)
    w, h = 48, 48
    cam = pt.camera_make((278.0, 273.0, -800.0 - 20 * 556.0), (278.0, 273.0, 0.0), 2.0, 1.0)
    s = make_scene(pt, p.objects, p.materials, gpu, wb)
    f = pt.Film(w, h, 3, device=gpu)
    rgb, st = pt.render(s, f, cam, 4, 8, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE, chunk=2)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    ref, rst = orc.render_sample(p.objects, p.materials, nodes, pt.camera_to_array(cam), w, h, f.rows, 4, 8, 3, 2,
                                 nthreads=8)
    assert np.array_equal(bits(rgb), bits(ref))
    assert st.rays == rst.rays and st.rays > w * h * 4


@pytest.mark.parametrize("name", ["cornell", "bunny_cornell"])
def test_wide_trace_near_axis_directions(pt, orc, gpu, wb, name):
    """The MIX plane arithmetic (wideHits<MIX>: fp16-denormal planes, scale s * 2^24 * inv) is exact
    while |inv| <= DevScene::mixLim; rays with a finite |1/d| component beyond it take the
    reference-order query (mixUnsafe), and so do rays with an exactly zero component (|inv| = inf:
    the decomposed planes would be NaN; since round 4, node visits guarded by
    test_gpu_zero_axis.py).  Axis-parallel and nearly axis-parallel rays (components 0, +-2^-100, +-2^-126, denormal)
    through the Cornell box's axis-aligned walls, from inside the box and aimed at vertices, keep
    the reference's hits bit for bit."""
    p = pt.Preset(name, 32, 32)
    objs = p.objects
    lo = objs["v"][:, :3].min(0)
    hi = objs["v"][:, :3].max(0)
    rng = np.random.default_rng(5)
    n = 8192
    o = (lo + (hi - lo) * rng.uniform(0.05, 0.95, (n, 3))).astype(np.float32)
    k = rng.integers(0, len(objs), n)
    tgt = objs["v"][k].reshape(-1, 3, 3)[np.arange(n), rng.integers(0, 3, n)]
    d = (tgt - o).astype(np.float32)
    tiny = np.array([0.0, 2.0 ** -100, -(2.0 ** -100), 2.0 ** -126, -(2.0 ** -140), 1e-42], np.float32)
    for i in range(n):   # one or two components replaced by a tiny value per ray
        ax = rng.permutation(3)[: 1 + (i % 2)]
        d[i, ax] = tiny[rng.integers(0, len(tiny), len(ax))]
    d[d.sum(1) == 0, 2] = 1.0
    rays = np.concatenate([o, d], 1).astype(np.float32)
    hits, st, ref, rst = trace_both(pt, orc, gpu, wb, objs, p.materials, rays)
    assert_hits_equal(hits, ref)
    assert ref["hit"].sum() > n // 2
    assert st.rays == len(rays)
