"""GPU parity tests: the HIP path (through the C ABI) against the CPU restatement (oracle/).

The kernels evaluate every expression in the reference's operation order with contraction
off, so the bar is BIT-EXACT for everything: LBVH topology and boxes, closest-hit records,
per-pixel RNG streams and rendered images (fp32 tolerance 0 ulp).  Full-size configurations
are covered through size-independent properties (determinism, stripe invariance, subsets of
rows checked against the oracle).
"""
import numpy as np
import pytest

from helpers import duplicate_centroids, random_rays, random_soup, rays_to_struct

pytestmark = pytest.mark.gpu


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
    h = g["hit"] == 1
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(bits(g[f][h]), bits(o[f][h]), err_msg=f)


SCENES = ["triangle_world", "random_world", "test_world", "rtiow", "cornell", "bunny_cornell"]


@pytest.mark.parametrize("name", SCENES)
def test_lbvh_matches_oracle(pt, orc, gpu, name):
    p = pt.Preset(name)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = s.download_bvh()
    ref = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    assert_nodes_equal(nodes, ref)
    assert s.bvh_info()["depth"] == orc.bvh_depth(ref, len(p.objects))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 1000])
def test_lbvh_small_and_duplicates(pt, orc, gpu, n):
    for objs, mats in (random_soup(n - n // 2, n // 2, seed=n), duplicate_centroids(n)):
        s = pt.Scene(objs, mats, device=gpu)
        assert_nodes_equal(s.download_bvh(), orc.build_lbvh(objs, orc.morton_keys(objs), tight=True))


def test_lbvh_large_soup(pt, orc, gpu):
    objs, mats = random_soup(150_000, 50_000, seed=7, spread=100.0)
    s = pt.Scene(objs, mats, device=gpu)
    assert_nodes_equal(s.download_bvh(), orc.build_lbvh(objs, orc.morton_keys(objs), tight=True))


@pytest.mark.parametrize("name", SCENES)
def test_trace_closest_matches_oracle(pt, orc, gpu, name):
    p = pt.Preset(name)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    ref_nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    lo = p.objects["v"][:, :3].min(0)
    hi = p.objects["v"][:, :3].max(0)
    center = np.clip((lo + hi) / 2, -1e3, 1e3)
    radius = float(min(np.linalg.norm(hi - lo), 3000.0)) * 0.75 + 1.0
    rays = random_rays(4096, seed=1, center=center, radius=radius, objects=p.objects)
    hits, st = s.trace(rays_to_struct(rays, pt.RAY_DTYPE))
    ref, rst = orc.trace(p.objects, ref_nodes, rays)
    assert_hits_equal(hits, ref)
    assert hits["hit"].sum() > 100
    assert st.node_visits == rst.node_visits and st.tri_tests == rst.tri_tests
    assert st.sphere_tests == rst.sphere_tests


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_trace_random_soup(pt, orc, gpu, seed):
    objs, mats = random_soup(3000, 500, seed=seed)
    s = pt.Scene(objs, mats, device=gpu)
    rays = random_rays(8192, seed=seed + 10, objects=objs)
    hits, _ = s.trace(rays_to_struct(rays, pt.RAY_DTYPE))
    ref, _ = orc.trace(objs, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), rays)
    assert_hits_equal(hits, ref)
    brute, _ = orc.trace(objs, None, rays, brute=True)   # BVH closest hit == brute force
    np.testing.assert_array_equal(ref["obj"], brute["obj"])


def test_trace_tmin_tmax_window(pt, orc, gpu):
    objs, mats = random_soup(500, 100, seed=3)
    s = pt.Scene(objs, mats, device=gpu)
    rays = random_rays(2048, seed=4, objects=objs)
    for tmin, tmax in ((0.001, 5.0), (2.0, 40.0), (0.0, np.inf)):
        hits, _ = s.trace(rays_to_struct(rays, pt.RAY_DTYPE), tmin, tmax)
        ref, _ = orc.trace(objs, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), rays, tmin, tmax)
        assert_hits_equal(hits, ref)


@pytest.mark.parametrize("parts", [1, 3])
def test_rng_streams_match_curand_init(pt, orc, gpu, parts):
    w, h = 97, 23
    for part in range(parts):
        f = pt.Film(w, h, seed=12345, device=gpu, stripe_height=4, n_parts=parts, part=part)
        np.testing.assert_array_equal(f.get_rng(), orc.film_states(12345, w, f.rows))


def test_rng_streams_far_pixels(pt, orc, gpu):
    """Pixel indices up to 1920*1080 exercise 21 jump matrices."""
    w, h = 1920, 1080
    f = pt.Film(w, h, seed=987654321987, device=gpu, stripe_height=8, n_parts=135, part=134)
    np.testing.assert_array_equal(f.get_rng(), orc.film_states(987654321987, w, f.rows))


def render_both(pt, orc, gpu, p, w, h, spp, depth, seed=1, parts=1, part=0, stripe=8):
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, seed, device=gpu, stripe_height=stripe, n_parts=parts, part=part)
    rgb, st = pt.render(s, f, p.camera, spp, depth)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    states = orc.film_states(seed, w, f.rows)
    ref, rst = orc.render(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, f.rows, spp, depth,
                          states, nthreads=8)
    return rgb, st, f.get_rng(), ref, rst, states, f


KERNELS = [("wide", "8", "16"), ("wavefront", "8", "16"), ("simple", "16", "24"), ("wide", "1", "1"),
           ("wide", "64", "64"), ("wavefront", "5", "50")]


@pytest.fixture(params=KERNELS, ids=lambda k: f"{k[0]}-L{k[1]}-S{k[2]}")
def kernel(request, monkeypatch):
    name, leaf, shade = request.param
    monkeypatch.setenv("PT_RENDER_KERNEL", name)
    monkeypatch.setenv("PT_LEAF_BATCH", leaf)
    monkeypatch.setenv("PT_SHADE_BATCH", shade)
    return request.param


@pytest.mark.parametrize("name,w,h,spp,depth", [
    ("rtiow", 64, 36, 4, 50),            # C1 scene: dielectric + metal + lambert spheres
    ("triangle_world", 80, 45, 4, 50),   # reference default scene
    ("random_world", 64, 36, 2, 50),
    ("test_world", 48, 27, 4, 50),
    ("cornell", 64, 64, 8, 8),           # C2 scene
    ("bunny_cornell", 96, 54, 2, 50),    # C3 scene
])
def test_render_bit_exact(pt, orc, gpu, kernel, name, w, h, spp, depth):
    p = pt.Preset(name, w, h)
    rgb, st, rng_after, ref, rst, ref_states, _ = render_both(pt, orc, gpu, p, w, h, spp, depth)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    np.testing.assert_array_equal(rng_after, ref_states)   # streams advanced identically
    assert st.rays == rst.rays and st.paths == rst.paths == w * h * spp
    # binary kernels: the same primitive tests in the same order (speculative traversal may visit
    # extra nodes); the wide tree tests its own set (same closest hits, tests/test_gpu_wide.py)
    if kernel[0] != "wide":
        assert st.tri_tests == rst.tri_tests and st.sphere_tests == rst.sphere_tests
    if kernel[0] == "simple":
        assert st.node_visits == rst.node_visits
    elif kernel[0] == "wavefront":
        assert st.node_visits >= rst.node_visits   # speculative traversal: a few extra binary nodes


@pytest.mark.parametrize("w,h,stripe", [(37, 19, 3), (50, 30, 8), (8, 8, 1)])
def test_render_stripes_assemble_to_full_frame(pt, orc, gpu, kernel, w, h, stripe):
    p = pt.Preset("rtiow", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    full, _ = pt.render(s, pt.Film(w, h, 5, device=gpu), p.camera, 3, 50)
    full = full.reshape(h, w, 3)
    for parts in (2, 3):
        img = np.zeros_like(full)
        for part in range(parts):
            f = pt.Film(w, h, 5, device=gpu, stripe_height=stripe, n_parts=parts, part=part)
            rgb, _ = pt.render(s, f, p.camera, 3, 50)
            img[f.rows] = rgb.reshape(f.n_rows, w, 3)
        np.testing.assert_array_equal(bits(img), bits(full))


def test_render_edge_cases(pt, orc, gpu, kernel):
    p = pt.Preset("rtiow", 16, 9)
    for depth in (0, 1):
        rgb, st, _, ref, _, _, _ = render_both(pt, orc, gpu, p, 16, 9, 2, depth)
        np.testing.assert_array_equal(bits(rgb), bits(ref))
        if depth == 0:
            assert st.rays == 0
    # single object (root is a leaf) and an empty-ish scene
    objs, mats = random_soup(0, 1, seed=1)
    objs["v"][0, :3] = [0, 0, -1]
    objs["v"][0, 3] = 0.5
    one = pt.Preset("rtiow", 16, 9)
    one.objects, one.materials = objs, mats
    rgb, _, _, ref, _, _, _ = render_both(pt, orc, gpu, one, 16, 9, 2, 5)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    # no objects at all (every path is the sky), and a 1x1 frame, in both RNG modes
    empty = pt.Preset("rtiow", 16, 9)
    empty.objects = empty.objects[:0]
    rgb, st, _, ref, _, _, _ = render_both(pt, orc, gpu, empty, 16, 9, 3, 50)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    assert st.rays == 16 * 9 * 3 and st.node_visits == 0
    for scene in (empty, pt.Preset("rtiow", 1, 1)):
        w, h = (16, 9) if scene is empty else (1, 1)
        s = pt.Scene(scene.objects, scene.materials, device=gpu)
        srgb, _ = pt.render(s, pt.Film(w, h, 4, device=gpu), scene.camera, 5, 50, rng=pt.RNG_SAMPLE, chunk=2)
        nodes = orc.build_lbvh(scene.objects, orc.morton_keys(scene.objects), tight=True) if len(scene.objects) \
            else np.zeros(0, pt.NODE_DTYPE)
        sref, _ = orc.render_sample(scene.objects, scene.materials, nodes, pt.camera_to_array(scene.camera), w, h,
                                    np.arange(h, dtype=np.int32), 5, 50, 4, 2, nthreads=2)
        np.testing.assert_array_equal(bits(srgb), bits(sref))


def test_render_continues_streams(pt, orc, gpu):
    """Two calls of spp=2 continue the per-pixel streams exactly like the reference's devStates."""
    w, h = 24, 16
    p = pt.Preset("cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, 9, device=gpu)
    a, _ = pt.render(s, f, p.camera, 2, 8)
    b, _ = pt.render(s, f, p.camera, 2, 8)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    states = orc.film_states(9, w, f.rows)
    cam = pt.camera_to_array(p.camera)
    ra, _ = orc.render(p.objects, p.materials, nodes, cam, w, h, f.rows, 2, 8, states, 4)
    rb, _ = orc.render(p.objects, p.materials, nodes, cam, w, h, f.rows, 2, 8, states, 4)
    np.testing.assert_array_equal(bits(a), bits(ra))
    np.testing.assert_array_equal(bits(b), bits(rb))
    assert not np.array_equal(a, b)


def test_full_size_c3_properties(pt, orc, gpu):
    """C3 frame size (1920x1080) at 1 spp: deterministic, finite, stripe-invariant, and a
    subset of rows bit-exact against the oracle."""
    p = pt.Preset("bunny_cornell")
    w, h = p.width, p.height
    s = pt.Scene(p.objects, p.materials, device=gpu)
    a, st = pt.render(s, pt.Film(w, h, 1, device=gpu), p.camera, 1, p.max_depth)
    b, _ = pt.render(s, pt.Film(w, h, 1, device=gpu), p.camera, 1, p.max_depth)
    np.testing.assert_array_equal(bits(a), bits(b))
    assert np.isfinite(a).all() and (a >= 0).all()
    assert st.paths == w * h and st.rays >= st.paths
    # rows 0, 540, 1079 through the oracle
    img = a.reshape(h, w, 3)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    rows = np.array([0, 540, 1079], np.int32)
    states = orc.film_states(1, w, rows)
    ref, _ = orc.render(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, rows, 1, p.max_depth,
                        states, 8)
    np.testing.assert_array_equal(bits(img[rows].reshape(-1, 3)), bits(ref))
    # 8-way stripes reproduce the full frame (the multi-GPU layout)
    img8 = np.zeros_like(img)
    for part in range(8):
        f = pt.Film(w, h, 1, device=gpu, stripe_height=8, n_parts=8, part=part)
        rgb, _ = pt.render(s, f, p.camera, 1, p.max_depth)
        img8[f.rows] = rgb.reshape(f.n_rows, w, 3)
    np.testing.assert_array_equal(bits(img8), bits(img))


def test_full_size_c5_bvh_and_trace(pt, orc, gpu):
    """C5 (1,043,312 triangles): GPU LBVH equals the oracle's, and closest hits agree."""
    p = pt.Preset("bunny_field")
    assert len(p.objects) == 1_043_312
    s = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = s.download_bvh()
    ref = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    assert_nodes_equal(nodes, ref)
    rays = random_rays(4096, seed=5, center=(278, 150, 280), radius=700, objects=p.objects)
    hits, _ = s.trace(rays_to_struct(rays, pt.RAY_DTYPE))
    rh, _ = orc.trace(p.objects, ref, rays)
    assert_hits_equal(hits, rh)


@pytest.mark.parametrize("kernel", ["wavefront", "wide"])
def test_c5_deep_tree_render_bit_exact(pt, orc, gpu, kernel):
    """C5's 1,043,312-triangle LBVH is deep (large LDS stack, leaf queue 4 in sample mode): a small
    frame of the C5 scene in both RNG modes, bit-exact against the oracle."""
    w, h, depth = 48, 27, 16
    p = pt.Preset("bunny_field", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    assert s.bvh_info()["depth"] >= 32   # depth + 1 > 32: the STACK = 48 instantiations
    k = pt.KERNEL_WAVEFRONT if kernel == "wavefront" else pt.KERNEL_WIDE
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    cam = pt.camera_to_array(p.camera)
    f = pt.Film(w, h, 3, device=gpu)
    rgb, st = pt.render(s, f, p.camera, 2, depth, kernel=k)
    ref, rst = orc.render(p.objects, p.materials, nodes, cam, w, h, f.rows, 2, depth, orc.film_states(3, w, f.rows),
                          nthreads=8)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    assert st.rays == rst.rays
    if kernel == "wavefront":   # the reference's primitive tests (the wide tree visits its own)
        assert st.tri_tests == rst.tri_tests
    srgb, sst = pt.render(s, f, p.camera, 5, depth, rng=pt.RNG_SAMPLE, chunk=2, kernel=k)
    sref, srst = orc.render_sample(p.objects, p.materials, nodes, cam, w, h, f.rows, 5, depth, 3, 2, nthreads=8)
    np.testing.assert_array_equal(bits(srgb), bits(sref))
    assert sst.rays == srst.rays
    if kernel == "wavefront":
        assert sst.tri_tests == srst.tri_tests


def test_device_output_pointer(gpu):
    """pt_render into a caller-owned device buffer (a torch tensor) on the caller's stream.
    Runs in a child process that imports torch BEFORE libpt.so, as bench.py does, so that both
    share one HIP runtime."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import ptamd as pt
p = pt.Preset("cornell", 32, 32)
s = pt.Scene(p.objects, p.materials, device=0)
host, _ = pt.render(s, pt.Film(32, 32, 3, device=0), p.camera, 2, 8)
out = torch.zeros((32 * 32, 3), dtype=torch.float32, device="cuda:0")
stream = torch.cuda.current_stream()
_, st = pt.render(s, pt.Film(32, 32, 3, device=0), p.camera, 2, 8, out=out.data_ptr(), stream=stream.cuda_stream)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy().view(np.uint32), host.view(np.uint32))
print("ok", st.rays)
"""
    import os
    pydir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-tracer-cuda-opengl_amd",
                         "python")
    r = subprocess.run([sys.executable, "-c", code, pydir], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_film_reset_and_explicit_kernels(pt, gpu):
    """pt_film_reset restores curand_init streams; both kernels (explicit options) give the
    identical frame from the same initial streams."""
    w, h = 96, 54
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, 4, device=gpu)
    init = f.get_rng()
    a, sa = pt.render(s, f, p.camera, 3, 50, kernel=pt.KERNEL_SIMPLE)
    f.reset()
    np.testing.assert_array_equal(f.get_rng(), init)
    b, sb = pt.render(s, f, p.camera, 3, 50, kernel=pt.KERNEL_WAVEFRONT, leaf_batch=9, shade_batch=33)
    np.testing.assert_array_equal(bits(a), bits(b))
    assert sa.rays == sb.rays and sa.tri_tests == sb.tri_tests
    f.reset()
    c, sc = pt.render(s, f, p.camera, 3, 50, kernel=pt.KERNEL_WIDE, leaf_batch=5, shade_batch=20)
    np.testing.assert_array_equal(bits(a), bits(c))
    assert sa.rays == sc.rays
    with pytest.raises(pt.PtError):
        pt.render(s, f, p.camera, 1, 5, kernel=7)


def test_lpt_tile_order_is_result_neutral(pt, gpu):
    """After a first launch the film launches tiles longest-first with raised priority for the
    head of the order; the frame must be bit-identical to the identity-order launch."""
    w, h = 160, 90
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, 21, device=gpu)
    frames = []
    for _ in range(3):   # 1st: identity order (no costs yet), 2nd/3rd: LPT from measured costs
        f.reset()
        rgb, st = pt.render(s, f, p.camera, 2, 50)
        frames.append(rgb.copy())
    for fr in frames[1:]:
        np.testing.assert_array_equal(bits(fr), bits(frames[0]))


# ---------------------------------------------------------------------------------------------
# Sample mode (PT_RNG_SAMPLE): Philox per pixel-sample, (tile, chunk) work units.
# ---------------------------------------------------------------------------------------------

def render_sample_both(pt, orc, gpu, p, w, h, spp, depth, seed, chunk, **kw):
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, seed, device=gpu, **kw)
    rgb, st = pt.render(s, f, p.camera, spp, depth, rng=pt.RNG_SAMPLE, chunk=chunk, kernel=pt.KERNEL_WAVEFRONT)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    ref, rst = orc.render_sample(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, f.rows, spp,
                                 depth, seed, chunk or max(16, -(-spp // 64)), nthreads=8)
    return rgb, st, ref, rst, s, f


@pytest.mark.parametrize("name,w,h,spp,depth,chunk", [
    ("rtiow", 64, 36, 5, 50, 2),             # ragged last chunk
    ("triangle_world", 80, 45, 4, 50, 0),    # default block (16) > spp: one block
    ("cornell", 64, 64, 9, 8, 4),
    ("bunny_cornell", 96, 54, 6, 50, 1),     # one sample per work unit
    ("bunny_cornell", 37, 19, 3, 50, 3),     # ragged tiles
])
def test_sample_mode_bit_exact(pt, orc, gpu, name, w, h, spp, depth, chunk, monkeypatch):
    for leaf, shade in (("8", "16"), ("1", "1")):
        monkeypatch.setenv("PT_LEAF_BATCH", leaf)
        monkeypatch.setenv("PT_SHADE_BATCH", shade)
        p = pt.Preset(name, w, h)
        rgb, st, ref, rst, s, f = render_sample_both(pt, orc, gpu, p, w, h, spp, depth, 11, chunk)
        np.testing.assert_array_equal(bits(rgb), bits(ref))
        assert st.rays == rst.rays and st.paths == rst.paths == w * h * spp
        assert st.tri_tests == rst.tri_tests and st.sphere_tests == rst.sphere_tests
        assert st.node_visits >= rst.node_visits   # speculative traversal
    # the ray-synchronous kernel: same frame, and exactly the reference's traversal order
    srgb, sst = pt.render(s, f, p.camera, spp, depth, rng=pt.RNG_SAMPLE, chunk=chunk, kernel=pt.KERNEL_SIMPLE)
    np.testing.assert_array_equal(bits(srgb), bits(ref))
    assert sst.node_visits == rst.node_visits and sst.tri_tests == rst.tri_tests
    # the 8-wide tree: same frame (its own visiting order, the reference's closest hits)
    for leaf, shade in (("24", "32"), ("1", "1")):
        monkeypatch.setenv("PT_LEAF_BATCH", leaf)
        monkeypatch.setenv("PT_SHADE_BATCH", shade)
        wrgb, wst = pt.render(s, f, p.camera, spp, depth, rng=pt.RNG_SAMPLE, chunk=chunk, kernel=pt.KERNEL_WIDE)
        np.testing.assert_array_equal(bits(wrgb), bits(ref))
        assert wst.rays == rst.rays


def test_sample_mode_stateless_and_stripes(pt, orc, gpu):
    """Sample mode is a pure function of (seed, pixel, sample): repeated calls agree, the film's
    XORWOW streams are untouched, and stripe partitions reassemble the full frame."""
    w, h, spp = 50, 30, 4
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, 3, device=gpu)
    init = f.get_rng()
    a, _ = pt.render(s, f, p.camera, spp, 50, rng=pt.RNG_SAMPLE, chunk=2)
    b, _ = pt.render(s, f, p.camera, spp, 50, rng=pt.RNG_SAMPLE, chunk=2)
    np.testing.assert_array_equal(bits(a), bits(b))
    np.testing.assert_array_equal(f.get_rng(), init)
    full = a.reshape(h, w, 3)
    for parts, stripe in ((2, 8), (3, 3)):
        img = np.zeros_like(full)
        for part in range(parts):
            fp = pt.Film(w, h, 3, device=gpu, stripe_height=stripe, n_parts=parts, part=part)
            rgb, _ = pt.render(s, fp, p.camera, spp, 50, rng=pt.RNG_SAMPLE, chunk=2)
            img[fp.rows] = rgb.reshape(fp.n_rows, w, 3)
        np.testing.assert_array_equal(bits(img), bits(full))
    # compat mode after sample mode still starts from the untouched streams
    c, _ = pt.render(s, f, p.camera, 1, 50)
    f.reset()
    d, _ = pt.render(s, f, p.camera, 1, 50)
    np.testing.assert_array_equal(bits(c), bits(d))


def test_sample_mode_options(pt, gpu):
    p = pt.Preset("cornell", 16, 16)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(16, 16, 1, device=gpu)
    with pytest.raises(pt.PtError):
        pt.render(s, f, p.camera, 1, 5, rng=5)
    with pytest.raises(pt.PtError):
        pt.render(s, f, p.camera, 1, 5, rng=pt.RNG_SAMPLE, kernel=9)
    a, _ = pt.render(s, f, p.camera, 2, 5, rng=pt.RNG_SAMPLE, kernel=pt.KERNEL_WAVEFRONT)
    b, _ = pt.render(s, f, p.camera, 2, 5, rng=pt.RNG_SAMPLE)
    c, _ = pt.render(s, f, p.camera, 2, 5, rng=pt.RNG_SAMPLE, kernel=pt.KERNEL_WIDE)
    np.testing.assert_array_equal(bits(a), bits(b))
    np.testing.assert_array_equal(bits(a), bits(c))
    _, st = pt.render(s, f, p.camera, 2, 0, rng=pt.RNG_SAMPLE)   # depth 0: no rays traced
    assert st.rays == 0


def test_sample_mode_full_size_c3_statistics(pt, orc, gpu):
    """C3 at full size: sample mode and compat mode are two estimates of the same image."""
    p = pt.Preset("bunny_cornell")
    w, h = p.width, p.height
    s = pt.Scene(p.objects, p.materials, device=gpu)
    a, sa = pt.render(s, pt.Film(w, h, 1, device=gpu), p.camera, 16, p.max_depth)
    b, sb = pt.render(s, pt.Film(w, h, 2, device=gpu), p.camera, 16, p.max_depth, rng=pt.RNG_SAMPLE, chunk=4)
    la = (a.astype(np.float64) ** 2).reshape(h // 40, 40, w // 40, 40, 3).mean(axis=(1, 3))
    lb = (b.astype(np.float64) ** 2).reshape(h // 40, 40, w // 40, 40, 3).mean(axis=(1, 3))
    assert np.abs(la - lb).mean() < 0.01 * max(la.mean(), 1e-3) + 0.002
    assert abs(sa.rays / sa.paths - sb.rays / sb.paths) < 0.02 * (sa.rays / sa.paths)
    # rows through the oracle
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    rows = np.array([3, 700], np.int32)
    ref, _ = orc.render_sample(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, rows, 16,
                               p.max_depth, 2, 4, 8)
    np.testing.assert_array_equal(bits(b.reshape(h, w, 3)[rows].reshape(-1, 3)), bits(ref))


def test_sample_mode_scheduling_is_result_neutral(pt, gpu):
    """Lanes take (pixel, block) tasks dynamically, in a tile order taken from the previous
    launch's costs; any schedule gives the identical frame."""
    w, h, spp = 96, 54, 40
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    f = pt.Film(w, h, 8, device=gpu)
    ref, _ = pt.render(s, f, p.camera, spp, 50, rng=pt.RNG_SAMPLE, chunk=4, flags=pt.IDENTITY_ORDER)
    for _ in range(3):   # 2nd and 3rd launch: longest tiles first
        rgb, st = pt.render(s, f, p.camera, spp, 50, rng=pt.RNG_SAMPLE, chunk=4)
        np.testing.assert_array_equal(bits(rgb), bits(ref))
    # a different spp after costs were measured: identical to a fresh film
    a, _ = pt.render(s, f, p.camera, 7, 50, rng=pt.RNG_SAMPLE, chunk=2)
    b, _ = pt.render(s, pt.Film(w, h, 8, device=gpu), p.camera, 7, 50, rng=pt.RNG_SAMPLE, chunk=2)
    np.testing.assert_array_equal(bits(a), bits(b))


@pytest.mark.parametrize("origin", [True, False])
@pytest.mark.parametrize("n", [1, 2, 5, 300, 20_000])
def test_device_morton_sort_matches_host_and_oracle(pt, orc, gpu, n, origin):
    """The device build (scene box, Morton codes, radix sort, leaf records) equals the host-keys
    build and the oracle's LBVH, node for node, with and without the origin in the bounds."""
    objs, mats = random_soup(n - n // 3, n // 3, seed=100 + n, spread=30.0)
    objs["v"][:, :3] += np.float32(50.0)   # off-origin: the origin flag changes the quantisation
    flags = pt.PT_BVH_ORIGIN_BOUNDS if origin else 0
    dev = pt.Scene(objs, mats, device=gpu, flags=flags)
    host = pt.Scene(objs, mats, device=gpu, flags=flags | pt.PT_BVH_HOST_KEYS)
    ref = orc.build_lbvh(objs, orc.morton_keys(objs, include_origin=origin), tight=True)
    assert_nodes_equal(dev.download_bvh(), ref)
    assert_nodes_equal(host.download_bvh(), ref)
    assert dev.bvh_info() == host.bvh_info()
    assert dev.build_ms > 0


def test_device_build_c5_faster_than_host_keys(pt, gpu):
    """C5 (1,043,312 triangles): the all-device build equals the host-keys build and is faster
    (wall time, host sort included)."""
    import time
    p = pt.Preset("bunny_field")
    s = pt.Scene(p.objects, p.materials, device=gpu, build=False)
    s.build_bvh()   # warm (code objects, allocations)
    t0 = time.perf_counter()
    s.build_bvh()
    t_dev = time.perf_counter() - t0
    a = s.download_bvh()
    t0 = time.perf_counter()
    s.build_bvh(pt.PT_BVH_ORIGIN_BOUNDS | pt.PT_BVH_HOST_KEYS)
    t_host = time.perf_counter() - t0
    assert_nodes_equal(s.download_bvh(), a)
    print(f"C5 LBVH build: device {t_dev * 1e3:.1f} ms, host keys {t_host * 1e3:.1f} ms")
    assert t_dev < t_host


@pytest.mark.parametrize("ways", [2, 4, 8])
@pytest.mark.parametrize("kname", ["wide", "wavefront"])
def test_compat_split_tiles_bit_exact(pt, orc, gpu, monkeypatch, kname, ways):
    """Compat mode's split tiles (PT_SPLIT_TILES / PT_SPLIT_WAYS: the longest tiles of the launch
    order run as `ways` waves of 64 / ways pixels each): launches after the first have a longest-
    first order and split; every launch's frame and advanced RNG streams equal the oracle's, with
    all tiles split and with only some (the frame's pixels rendered exactly once)."""
    monkeypatch.setenv("PT_RENDER_KERNEL", kname)
    monkeypatch.setenv("PT_SPLIT_WAYS", str(ways))
    w, h, spp, depth = 72, 40, 3, 50
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    f = pt.Film(w, h, 4, device=gpu)
    ref_states = orc.film_states(4, w, f.rows)   # (advanced by the render below)
    ref, rst = orc.render(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, f.rows, spp, depth,
                          ref_states, nthreads=8)
    ntiles = ((w + 7) // 8) * ((h + 7) // 8)
    for split in (str(ntiles), "7", "0"):
        monkeypatch.setenv("PT_SPLIT_TILES", split)
        for _ in range(2):   # (the first launch of a film has no order yet; later ones split)
            f.reset()
            rgb, st = pt.render(s, f, p.camera, spp, depth)
            np.testing.assert_array_equal(bits(rgb), bits(ref))
            assert st.rays == rst.rays and st.paths == w * h * spp
            np.testing.assert_array_equal(f.get_rng(), ref_states)


@pytest.mark.parametrize("crit,lanes", [("1", "1"), ("100", "8"), ("100000", "64"), ("37", "3")])
def test_compat_critical_pixels_bit_exact(pt, orc, gpu, monkeypatch, crit, lanes):
    """Compat mode's critical pixels (the wide kernel on shallow trees, long paths): launches after
    the first take the previous launch's PT_CRIT_PIXELS longest per-pixel chains out of the tile
    waves and run them first, PT_CRIT_LANES per wave, each lane tracing its rays in one per-lane
    loop.  Every launch's frame, advanced RNG streams and counters equal the oracle's -- with one
    critical pixel, some, every pixel of the frame, and ragged waves."""
    monkeypatch.setenv("PT_CRIT_PIXELS", crit)
    monkeypatch.setenv("PT_CRIT_LANES", lanes)
    w, h, spp, depth = 72, 40, 3, 50
    p = pt.Preset("bunny_cornell", w, h)
    s = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    f = pt.Film(w, h, 6, device=gpu)
    ref_states = orc.film_states(6, w, f.rows)
    ref, rst = orc.render(p.objects, p.materials, nodes, pt.camera_to_array(p.camera), w, h, f.rows, spp, depth,
                          ref_states, nthreads=8)
    for _ in range(3):   # (the first launch measures the chains; later ones run the critical pixels first)
        f.reset()
        rgb, st = pt.render(s, f, p.camera, spp, depth, kernel=pt.KERNEL_WIDE)
        np.testing.assert_array_equal(bits(rgb), bits(ref))
        assert st.rays == rst.rays and st.paths == w * h * spp
        assert st.tri_tests > 0 and st.node_visits > 0   # (the wide tree's own counts, not the oracle's)
        np.testing.assert_array_equal(f.get_rng(), ref_states)
    # accumulating frames (raw sums through the resolve pass) and 8-bit output take the same path
    f.reset()
    f.clear()
    a, _ = pt.render(s, f, p.camera, spp, depth, kernel=pt.KERNEL_WIDE, accumulate=True)
    np.testing.assert_array_equal(bits(a), bits(ref))


@pytest.mark.parametrize("spp,chunk", [(128, 16), (96, 4)])
def test_sample_mode_repeated_launches_bit_exact(pt, orc, gpu, spp, chunk):
    """Sample mode on several launches of one film (the first measures tile costs, then frames
    without them and, every 8th, with them again): every frame of the wide kernel equals the oracle."""
    w, h, depth = 48, 40, 50
    p = pt.Preset("bunny_cornell", w, h)
    rgb, st, ref, rst, s, f = render_sample_both(pt, orc, gpu, p, w, h, spp, depth, 5, chunk)
    np.testing.assert_array_equal(bits(rgb), bits(ref))
    for _ in range(9):
        again, ast = pt.render(s, f, p.camera, spp, depth, rng=pt.RNG_SAMPLE, chunk=chunk, kernel=pt.KERNEL_WIDE)
        np.testing.assert_array_equal(bits(again), bits(ref))
        assert ast.rays == rst.rays
